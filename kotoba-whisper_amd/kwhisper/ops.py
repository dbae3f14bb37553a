"""Torch-tensor front end of the kwhisper C ABI, through the PyTorch-ROCm custom ops ``torch.ops.kw.*``.

Every launch goes through a ``torch.ops.kw`` operator (``csrc/torch_ops.cpp``, SURVEY.md §8b: "Torch custom
ops wrap the ABI"), which fills the C ABI's argument block and launches on torch's current HIP stream, so
the kernels are ordinary torch ops to the dispatcher, to ``torch.cuda.graph`` capture and to
``torch.compile`` (fake implementations are registered: every op mutates its outputs and returns nothing).
Tensors are plumbing only (device memory + stream); all arithmetic happens in the HIP kernels of
``libkwhisper.so``.  The plan classes (``GemmPlan``, ``DecLinearPlan``, ``SamplerPlan``, ``BeamStepPlan``)
validate once and keep the op arguments, so decode steps replay without re-validation.

``set_backend("ctypes")`` routes the same calls through the ctypes binding of the C ABI instead (used by
the test that holds the two paths bitwise equal); there is no CPU or torch fallback on either path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib as L

_DT = {torch.float32: L.KW_DT_F32, torch.bfloat16: L.KW_DT_BF16}
_BACKEND = "torch"


def set_backend(name: str) -> str:
    """Select "torch" (torch.ops.kw, the default) or "ctypes" (the C ABI bound directly); returns the old one."""
    global _BACKEND
    if name not in ("torch", "ctypes"):
        raise ValueError("backend must be 'torch' or 'ctypes'")
    old, _BACKEND = _BACKEND, name
    return old


def backend() -> str:
    return _BACKEND


def _kw():
    """The torch.ops.kw namespace (loads libkwhisper_torch.so once; raises if it is missing)."""
    return L.load_torch_ops()


def _lib():
    return L.load()


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dt(t: torch.Tensor) -> int:
    try:
        return _DT[t.dtype]
    except KeyError:
        raise ValueError(f"unsupported dtype {t.dtype}; expected float32 or bfloat16") from None


def _cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("kwhisper ops take device (cuda) tensors")


def _ws_bytes(kind: str, *dims) -> int:
    if _BACKEND == "torch":
        return int(_kw().workspace_bytes(kind, [int(d) for d in dims]))
    fn = {"dec_linear": "kw_dec_linear_workspace_bytes", "packed_weight": "kw_packed_weight_bytes",
          "self_attn": "kw_self_attn_workspace", "cross_attn": "kw_cross_attn_workspace",
          "greedy_step": "kw_greedy_step_workspace", "beam_logprobs": "kw_beam_logprobs_workspace",
          "lm_greedy": "kw_dec_lm_greedy_workspace",
          "qkv_self": "kw_dec_qkv_self_workspace", "xq_cross": "kw_dec_xq_cross_workspace",
          "qkv_self_status": "kw_dec_qkv_self_status_offset", "xq_cross_status": "kw_dec_xq_cross_status_offset",
          "cross_attn_status": "kw_cross_attn_status_offset"}[kind]
    return int(getattr(_lib(), fn)(*dims))


def log_mel(audio: torch.Tensor, mel_filters: torch.Tensor, out: torch.Tensor | None = None,
            workspace: torch.Tensor | None = None) -> torch.Tensor:
    """audio (B, n) f32, n % 160 == 0 -> (B, n_mels, n // 160) f32 log-mel."""
    _cuda(audio, mel_filters)
    if audio.dim() != 2 or audio.dtype != torch.float32 or audio.stride(1) != 1:
        raise ValueError("audio must be a (B, n_samples) float32 tensor with unit inner stride")
    if mel_filters.dim() != 2 or mel_filters.shape[0] != 201 or not mel_filters.is_contiguous():
        raise ValueError("mel_filters must be a contiguous (201, n_mels) float32 tensor")
    b, n = audio.shape
    n_mels = mel_filters.shape[1]
    if out is None:
        out = torch.empty((b, n_mels, n // 160), device=audio.device, dtype=torch.float32)
    if workspace is None:
        workspace = torch.empty((max(b, 1),), device=audio.device, dtype=torch.int32)
    if _BACKEND == "torch":
        _kw().log_mel(audio, mel_filters, out, workspace)
    else:
        L.check(_lib().kw_log_mel(_p(audio), b, n, audio.stride(0), _p(mel_filters), n_mels, _p(out), _p(workspace),
                                  _s()), "kw_log_mel")
    return out


def mel_to_time_major(mel: torch.Tensor, c_pad: int, dtype: torch.dtype, out: torch.Tensor | None = None):
    _cuda(mel)
    b, c, t = mel.shape
    if out is None:
        out = torch.empty((b, t + 2, c_pad), device=mel.device, dtype=dtype)
    mel = mel.contiguous()
    if _BACKEND == "torch":
        _kw().mel_to_time_major(mel, c_pad, out)
    else:
        L.check(_lib().kw_mel_to_time_major(_p(mel), b, c, t, c_pad, _p(out), _DT[dtype], _s()), "kw_mel_to_time_major")
    return out


def layernorm(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, out: torch.Tensor,
              delta: torch.Tensor | None = None):
    """out = LayerNorm(x); with ``delta`` (bf16, x's shape) x += delta first, in place.  x is the residual
    stream: f32 (kw_layernorm) or bf16 (kw_layernorm_bf16res, the sum rounded to bf16)."""
    _cuda(x, gamma, beta, out, delta)
    if x.dtype not in (torch.float32, torch.bfloat16) or not x.is_contiguous():
        raise ValueError("layernorm input must be contiguous float32 or bfloat16")
    if delta is not None and (delta.dtype != torch.bfloat16 or delta.numel() != x.numel() or not delta.is_contiguous()):
        raise ValueError("layernorm delta must be a contiguous bf16 tensor of x's size")
    if _BACKEND == "torch":
        _kw().layernorm(x, gamma, beta, float(eps), out, delta)
        return out
    dim = x.shape[-1]
    rows = x.numel() // dim
    if x.dtype == torch.bfloat16:
        L.check(_lib().kw_layernorm_bf16res(_p(x), rows, dim, _p(gamma), _p(beta), eps, _p(out), _dt(out), _p(delta),
                                            _s()), "kw_layernorm_bf16res")
    else:
        L.check(_lib().kw_layernorm(_p(x), rows, dim, _p(gamma), _p(beta), eps, _p(out), _dt(out), _p(delta), _s()),
                "kw_layernorm")
    return out


class GemmPlan:
    """A pre-built ``kw_gemm`` call: C = epilogue(A . W^T + bias)."""

    def __init__(self, A, W, C, M, N, K, *, bias=None, lda=None, a_rows_per_batch=0, a_batch_stride=0,
                 ldc=None, c_rows_per_batch=0, c_batch_stride=0, epilogue=L.KW_EPI_STORE, gelu=False,
                 scale=1.0, scale_cols=0, row_add=None, row_add_period=0, hs_seq=0, hs_heads=0, hs_head_dim=0,
                 dtype=None, a_offset=0, c_offset=0):
        _cuda(A, W, C, bias, row_add)
        if bias is not None and bias.dtype != torch.float32:
            raise ValueError("bias must be float32")
        if row_add is not None and row_add.dtype != torch.float32:
            raise ValueError("row_add must be float32")
        lda = K if lda is None else lda
        ldc = N if ldc is None else ldc
        self._keep = (A, W, C, bias, row_add)
        # torch.ops.kw.gemm arguments
        self._geo = [a_offset, lda, a_rows_per_batch, a_batch_stride, c_offset, ldc, c_rows_per_batch, c_batch_stride,
                     M, N, K, epilogue, int(bool(gelu)), scale_cols, row_add_period, hs_seq, hs_heads, hs_head_dim]
        self._targs = (A, W, bias, C, row_add, self._geo, float(scale), -1 if dtype is None else _DT[dtype])
        # the same call as a C argument block (ctypes backend)
        a = L.GemmArgs()
        a.dtype = _dt(W) if dtype is None else _DT[dtype]
        a.c_dtype = _dt(C)
        a.A = A.data_ptr() + a_offset * A.element_size()
        a.lda, a.a_rows_per_batch, a.a_batch_stride = lda, a_rows_per_batch, a_batch_stride
        a.W = W.data_ptr()
        a.bias = bias.data_ptr() if bias is not None else None
        a.C = C.data_ptr() + c_offset * C.element_size()
        a.ldc, a.c_rows_per_batch, a.c_batch_stride = ldc, c_rows_per_batch, c_batch_stride
        a.M, a.N, a.K = M, N, K
        a.epilogue = epilogue
        a.gelu = int(bool(gelu))
        a.scale = float(scale)
        a.scale_cols = scale_cols
        a.row_add = row_add.data_ptr() if row_add is not None else None
        a.row_add_period = row_add_period
        a.hs_seq, a.hs_heads, a.hs_head_dim = hs_seq, hs_heads, hs_head_dim
        self.args = a
        self._ref = ctypes.byref(a)

    def __call__(self):
        if _BACKEND == "torch":
            _kw().gemm(*self._targs)
        else:
            L.check(_lib().kw_gemm(self._ref, _s()), "kw_gemm")


def dec_linear_workspace_bytes(N: int, K: int) -> int:
    return _ws_bytes("dec_linear", N, K)


class DecLinearPlan:
    """A pre-built ``kw_dec_linear`` call (decode-step linear over packed weights).

    ``x``: bf16 [M][ldx] activations (x_offset elements from the start); ``ln`` = (eps, colsum f32 [N])
    fuses the LayerNorm of x's rows (gamma/beta folded into W/bias by the caller, colsum = row sums of
    the folded bf16 weight: ``ln_colsum``); STORE writes ``C`` (f32 or bf16, ldc); RESID updates
    ``resid`` = (h f32, hb bf16 mirror, ldh, row offset)."""

    def __init__(self, x, W, M, N, K, *, ldx=None, x_offset=0, ln=None, bias=None, C=None, ldc=None, c_offset=0,
                 gelu=False, scale=1.0, scale_cols=0, resid=None, workspace=None, tag=None):
        _cuda(x, W, bias, C, workspace)
        self.tag = tag  # a name for per-kernel timing (bench.py), no effect on the call
        if x.dtype != torch.bfloat16 or W.dtype != torch.bfloat16:
            raise ValueError("kw_dec_linear takes bf16 activations and packed bf16 weights")
        if bias is not None and bias.dtype != torch.float32:
            raise ValueError("bias must be float32")
        ldx = K if ldx is None else ldx
        a = L.DecLinearArgs()
        keep = [x, W, bias, C, workspace]
        a.x = x.data_ptr() + x_offset * 2
        a.ldx = ldx
        colsum, eps = None, 0.0
        if ln is not None:
            eps, colsum = ln
            _cuda(colsum)
            if colsum.dtype != torch.float32 or colsum.numel() < N:
                raise ValueError("ln colsum must be float32 [N]")
            a.ln = 1
            a.ln_eps = float(eps)
            a.ln_colsum = colsum.data_ptr()
            keep.append(colsum)
        a.W = W.data_ptr()
        a.bias = bias.data_ptr() if bias is not None else None
        h = hb = None
        row0 = ldh = 0
        if resid is not None:
            h, hb, ldh, row0 = resid
            _cuda(h, hb)
            if h.dtype != torch.float32 or hb.dtype != torch.bfloat16:
                raise ValueError("RESID needs an f32 residual and a bf16 mirror")
            a.epilogue = L.KW_EPI_RESID
            a.h = h.data_ptr() + row0 * ldh * 4
            a.hb = hb.data_ptr() + row0 * ldh * 2
            a.ldh = ldh
            keep += [h, hb]
            C = None
        else:
            if C is None:
                raise ValueError("STORE needs C")
            a.epilogue = L.KW_EPI_STORE
            ldc = N if ldc is None else ldc
            a.C = C.data_ptr() + c_offset * C.element_size()
            a.ldc = ldc
            a.c_dtype = _dt(C)
        a.gelu = int(bool(gelu))
        a.scale = float(scale)
        a.scale_cols = scale_cols
        a.M, a.N, a.K = M, N, K
        need = dec_linear_workspace_bytes(N, K)
        if workspace is None:
            workspace = torch.zeros((need + 3) // 4, device=W.device, dtype=torch.float32)
            keep.append(workspace)
        if workspace.numel() * workspace.element_size() < need:
            raise ValueError("kw_dec_linear workspace too small")
        a.workspace = workspace.data_ptr()
        a.ws_bytes = workspace.numel() * workspace.element_size()
        self._keep = tuple(keep)
        geo = [x_offset, ldx, 1 if ln is not None else 0, c_offset, 0 if C is None else (ldc or N), int(bool(gelu)),
               scale_cols, row0, ldh, M, N, K]
        self._targs = (x, W, bias, colsum, C, h, hb, workspace, geo, float(eps), float(scale))
        self.args = a
        self._ref = ctypes.byref(a)

    def __call__(self):
        if _BACKEND == "torch":
            _kw().dec_linear(*self._targs)
        else:
            L.check(_lib().kw_dec_linear(self._ref, _s()), "kw_dec_linear")


def ln_colsum(W: torch.Tensor) -> torch.Tensor:
    """f32 [N] row sums of a bf16 [N][K] weight (the values kw_dec_linear multiplies), accumulated in f64."""
    return W.double().sum(1).float().contiguous()


def pack_weight(W: torch.Tensor) -> torch.Tensor:
    """[N][K] bf16 -> packed 16x32-fragment layout for kw_dec_linear."""
    _cuda(W)
    if W.dtype != torch.bfloat16 or W.dim() != 2 or not W.is_contiguous():
        raise ValueError("pack_weight expects a contiguous 2-D bfloat16 tensor")
    n, k = W.shape
    nbytes = _ws_bytes("packed_weight", n, k)
    out = torch.empty((nbytes // 2,), device=W.device, dtype=torch.bfloat16)
    if _BACKEND == "torch":
        _kw().pack_weight(W, out)
    else:
        L.check(_lib().kw_pack_weight(_p(W), n, k, _p(out), _s()), "kw_pack_weight")
    return out


KW_ATTN_Q_LOG2 = 0x100


def attention(qkv: torch.Tensor, B: int, H: int, T: int, hd: int, out: torch.Tensor, q_log2: bool = False):
    """Encoder self-attention; ``q_log2``: q also carries log2(e) (bf16 only; kw_attention's KW_ATTN_Q_LOG2)."""
    _cuda(qkv, out)
    if qkv.numel() != 3 * B * H * T * hd or out.numel() != B * T * H * hd or qkv.dtype != out.dtype:
        raise ValueError("attention: qkv must hold [3][B][H][T][hd] and out [B][T][H*hd] of one dtype")
    flags = KW_ATTN_Q_LOG2 if q_log2 else 0
    if _BACKEND == "torch":
        _kw().attention(qkv, B, H, T, hd, out, flags)
    else:
        L.check(_lib().kw_attention(_dt(qkv) | flags, _p(qkv), B, H, T, hd, _p(out), _s()), "kw_attention")
    return out


def embed(ids, B, q_len, cur_len, tok_emb, pos_emb, h, hb=None):
    """Decoder embedding into the f32 residual h (and its bf16 mirror hb for the bf16 engine)."""
    _cuda(ids, cur_len, tok_emb, pos_emb, h, hb)
    if _BACKEND == "torch":
        _kw().embed(ids, B, q_len, cur_len, tok_emb, pos_emb, h, hb)
    else:
        L.check(_lib().kw_embed(_dt(tok_emb), _p(ids), ids.stride(0), B, q_len, _p(cur_len), _p(tok_emb), _p(pos_emb),
                                tok_emb.shape[1], _p(h), _p(hb), _s()), "kw_embed")


def self_attn_workspace_bytes(B, H, t_max) -> int:
    return _ws_bytes("self_attn", B, H, t_max)


def self_attn_step(qkv, B, q_len, H, hd, k_cache, v_cache, t_max, cur_len, out, workspace=None, bp=None):
    """Static-cache self-attention; q_len == 1 needs a zero-filled ``workspace`` (self_attn_workspace_bytes);
    ``bp``: beam-search slot table [B][>= t_max] int32 (q_len == 1)."""
    _cuda(qkv, k_cache, v_cache, cur_len, out, workspace, bp)
    if _BACKEND == "torch":
        _kw().self_attn_step(qkv, B, q_len, H, hd, k_cache, v_cache, t_max, cur_len, out, workspace, bp)
        return
    nb = workspace.numel() * workspace.element_size() if workspace is not None else 0
    L.check(_lib().kw_self_attn_step(_dt(qkv), _p(qkv), B, q_len, H, hd, _p(k_cache), _p(v_cache), t_max,
                                     _p(cur_len), _p(bp), bp.stride(0) if bp is not None else 0, _p(out),
                                     _p(workspace), nb, _s()), "kw_self_attn_step")


def qkv_self_workspace_bytes(M, d) -> int:
    return _ws_bytes("qkv_self", M, d)


def qkv_self_supported(M, d, H) -> bool:
    """Whether kw_dec_qkv_self covers the shape (M <= 32, d = 64 H <= 1280)."""
    return bool(_lib().kw_dec_qkv_self_supported(int(M), int(d), int(H)))


class QkvSelfPlan:
    """A pre-built ``kw_dec_qkv_self`` call: LayerNorm-fused QKV projection + self-attention step of one decode
    step in one launch (kw_dec_linear(qkv) then kw_self_attn_step: caches bitwise, attention within bf16 rounding).  ``x``: hb [M][ldx] bf16;
    ``W`` packed (gamma folded), ``ln`` = (eps, colsum [3d]), ``bias`` f32 [3d]; caches one layer's
    [M][H][t_max][64]; ``cur_len`` device int32 (L <= 256); ``out`` attn [M][d] bf16; ``workspace`` zero-filled
    (qkv_self_workspace_bytes)."""

    def __init__(self, x, W, M, d, H, *, ln, bias, scale, k_cache, v_cache, t_max, cur_len, out, workspace, ldx=None,
                 tag="qkv_self"):
        _cuda(x, W, bias, k_cache, v_cache, cur_len, out, workspace)
        eps, colsum = ln
        _cuda(colsum)
        if x.dtype != torch.bfloat16 or W.dtype != torch.bfloat16 or out.dtype != torch.bfloat16:
            raise ValueError("kw_dec_qkv_self takes bf16 activations, packed bf16 weights and a bf16 output")
        ldx = d if ldx is None else ldx
        if workspace.numel() * workspace.element_size() < qkv_self_workspace_bytes(M, d):
            raise ValueError("kw_dec_qkv_self workspace too small")
        self.tag = tag
        a = L.QkvSelfArgs()
        a.x, a.ldx, a.ln_eps, a.ln_colsum = x.data_ptr(), ldx, float(eps), colsum.data_ptr()
        a.W, a.bias, a.scale = W.data_ptr(), bias.data_ptr() if bias is not None else None, float(scale)
        a.M, a.d, a.H = M, d, H
        a.k_cache, a.v_cache, a.t_max, a.cur_len = k_cache.data_ptr(), v_cache.data_ptr(), t_max, cur_len.data_ptr()
        a.out, a.workspace = out.data_ptr(), workspace.data_ptr()
        a.ws_bytes = workspace.numel() * workspace.element_size()
        self._a = a
        self._ref = ctypes.byref(a)
        self._keep = (x, W, bias, colsum, k_cache, v_cache, cur_len, out, workspace)
        self._targs = (x, W, bias, colsum, k_cache, v_cache, cur_len, out, workspace, [ldx, M, d, H, t_max],
                       float(eps), float(scale))

    def __call__(self):
        if _BACKEND == "torch":
            _kw().dec_qkv_self(*self._targs)
        else:
            L.check(_lib().kw_dec_qkv_self(self._ref, _s()), "kw_dec_qkv_self")


def xq_cross_workspace_bytes(M, d, H, S) -> int:
    return _ws_bytes("xq_cross", M, d, H, S)


def xq_cross_supported(M, d, H, S) -> bool:
    """Whether kw_dec_xq_cross can run here: the shape is one it covers (M <= 32, d = 64 H <= 1280, S whose
    chunks hold 225..256 keys)."""
    return bool(_lib().kw_dec_xq_cross_supported(int(M), int(d), int(H), int(S)))


def cross_attn_pair_kernel(rows, S, fused=False) -> bool:
    """Whether a bf16 one-row cross-attention of ``rows`` (row, head) pairs runs as one workgroup per pair
    (cross_attn_row_kernel) rather than per (pair, chunk) -- kernel naming for profiles; results are equal."""
    return bool(_lib().kw_cross_attn_pair_kernel(int(rows), int(S), int(bool(fused))))


class XqCrossPlan:
    """A pre-built ``kw_dec_xq_cross`` call: the LayerNorm-fused cross-attention query projection and the
    cross-attention step (q_len 1) in one launch (bitwise kw_dec_linear(xq) then kw_cross_attn_step).  ``x``: hb [M][ldx] bf16; ``W`` packed (gamma folded), ``ln`` = (eps, colsum [d]), ``bias``
    f32 [d]; ``k`` / ``v`` one layer's [M][H][S][64]; ``out`` attn [M][d] bf16; ``workspace`` zero-filled
    (xq_cross_workspace_bytes)."""

    def __init__(self, x, W, M, d, H, *, ln, bias, scale, k, v, S, out, workspace, ldx=None, tag="xq_cross"):
        _cuda(x, W, bias, k, v, out, workspace)
        eps, colsum = ln
        _cuda(colsum)
        if any(t.dtype != torch.bfloat16 for t in (x, W, k, v, out)):
            raise ValueError("kw_dec_xq_cross takes bf16 activations, packed bf16 weights, bf16 K / V and output")
        ldx = d if ldx is None else ldx
        if workspace.numel() * workspace.element_size() < xq_cross_workspace_bytes(M, d, H, S):
            raise ValueError("kw_dec_xq_cross workspace too small")
        self.tag = tag
        a = L.XqCrossArgs()
        a.x, a.ldx, a.ln_eps, a.ln_colsum = x.data_ptr(), ldx, float(eps), colsum.data_ptr()
        a.W, a.bias, a.scale = W.data_ptr(), bias.data_ptr() if bias is not None else None, float(scale)
        a.M, a.d, a.H = M, d, H
        a.k, a.v, a.S = k.data_ptr(), v.data_ptr(), S
        a.out, a.workspace = out.data_ptr(), workspace.data_ptr()
        a.ws_bytes = workspace.numel() * workspace.element_size()
        self._a = a
        self._ref = ctypes.byref(a)
        self._keep = (x, W, bias, colsum, k, v, out, workspace)
        self._targs = (x, W, bias, colsum, k, v, out, workspace, [ldx, M, d, H, S], float(eps), float(scale))

    def __call__(self):
        if _BACKEND == "torch":
            _kw().dec_xq_cross(*self._targs)
        else:
            L.check(_lib().kw_dec_xq_cross(self._ref, _s()), "kw_dec_xq_cross")


def cross_attn_workspace_bytes(B, q_len, H, hd, S) -> int:
    return _ws_bytes("cross_attn", B, q_len, H, hd, S)


def status_offset(kind: str, *dims) -> int:
    """Byte offset of the int32 hand-off status word inside the workspace of ``kind`` ("qkv_self",
    "xq_cross", "cross_attn"; the workspace's own dimensions).  The word after it (qkv_self, xq_cross) is the
    fault-injection word (include/kwhisper.h)."""
    return _ws_bytes(f"{kind}_status", *dims)


def cross_attn_step(q, B, q_len, H, hd, k, v, S, out, workspace):
    _cuda(q, k, v, out, workspace)
    if _BACKEND == "torch":
        _kw().cross_attn_step(q, B, q_len, H, hd, k, v, S, out, workspace)
        return
    L.check(_lib().kw_cross_attn_step(_dt(q), _p(q), B, q_len, H, hd, _p(k), _p(v), S, _p(out), _p(workspace),
                                      workspace.numel() * workspace.element_size(), _s()), "kw_cross_attn_step")


def beam_logprobs_workspace_bytes(R: int) -> int:
    return _ws_bytes("beam_logprobs", R)


def greedy_step_workspace_bytes(B: int) -> int:
    return _ws_bytes("greedy_step", B)


class SamplerPlan:
    """Pre-built ``kw_greedy_step`` call (processors + argmax + stopping on device)."""

    def __init__(self, logits, suppress_mask, begin_suppress, ids, cur_len, unfinished, counter, n_unfinished, *,
                 return_timestamps, ts_begin, no_ts_id, eos_id, pad_id, max_initial_ts, max_length, begin_index,
                 scores_out=None, workspace=None):
        _cuda(logits, suppress_mask, begin_suppress, ids, cur_len, unfinished, counter, n_unfinished, scores_out,
              workspace)
        self._keep = (logits, suppress_mask, begin_suppress, ids, cur_len, unfinished, counter, n_unfinished, scores_out,
                      workspace)
        mit = -1 if max_initial_ts is None else max_initial_ts
        cfg = [int(bool(return_timestamps)), ts_begin, no_ts_id, eos_id, pad_id, mit, max_length, begin_index]
        self._targs = (logits, suppress_mask, begin_suppress, ids, cur_len, unfinished, counter, n_unfinished,
                       scores_out, workspace, cfg)
        a = L.SamplerArgs()
        a.logits = logits.data_ptr()
        a.B, a.V = logits.shape
        a.suppress_mask = suppress_mask.data_ptr()
        a.begin_suppress = begin_suppress.data_ptr() if begin_suppress is not None else None
        a.n_begin_suppress = begin_suppress.numel() if begin_suppress is not None else 0
        a.return_timestamps = int(bool(return_timestamps))
        a.ts_begin, a.no_ts_id, a.eos_id, a.pad_id = ts_begin, no_ts_id, eos_id, pad_id
        a.max_initial_ts = mit
        a.ids = ids.data_ptr()
        a.ids_stride = ids.stride(0)
        a.cur_len = cur_len.data_ptr()
        a.max_length = max_length
        a.begin_index = begin_index
        a.unfinished = unfinished.data_ptr()
        a.counter = counter.data_ptr()
        a.n_unfinished = n_unfinished.data_ptr()
        a.scores_out = scores_out.data_ptr() if scores_out is not None else None
        a.workspace = workspace.data_ptr() if workspace is not None else None
        a.ws_bytes = workspace.numel() * workspace.element_size() if workspace is not None else 0
        self.args = a
        self._ref = ctypes.byref(a)

    def __call__(self):
        if _BACKEND == "torch":
            _kw().greedy_step(*self._targs)
        else:
            L.check(_lib().kw_greedy_step(self._ref, _s()), "kw_greedy_step")


def lm_greedy_workspace_bytes(B: int, V: int) -> int:
    return _ws_bytes("lm_greedy", B, V)


def lm_greedy_supported(B: int, V: int, d: int) -> bool:
    """Whether kw_dec_lm_greedy covers the shape (B <= 32 rows, the persistent LM head's geometry)."""
    return bool(_lib().kw_dec_lm_greedy_supported(int(B), int(V), int(d)))


class LmGreedyPlan:
    """A pre-built ``kw_dec_lm_greedy`` call: the LM head (final LayerNorm folded, as the ``DecLinearPlan`` with
    ``ln`` it replaces) and the greedy step without timestamps (as ``SamplerPlan``) in one launch.  ``x``: hb
    [M][ldx] bf16 (x_offset elements in); ``logits``: optional f32 [M][V] (None: not stored); ``workspace``
    zero-filled (lm_greedy_workspace_bytes); the device state (ids, cur_len, unfinished, n_unfinished) is the
    sampler's."""

    def __init__(self, x, W, M, N, K, *, ln, bias, suppress_mask, begin_suppress, ids, cur_len, unfinished,
                 n_unfinished, eos_id, pad_id, max_length, begin_index, workspace, logits=None, ldx=None, x_offset=0,
                 tag="lm_greedy"):
        eps, colsum = ln
        _cuda(x, W, bias, colsum, logits, suppress_mask, begin_suppress, ids, cur_len, unfinished, n_unfinished,
              workspace)
        if x.dtype != torch.bfloat16 or W.dtype != torch.bfloat16:
            raise ValueError("kw_dec_lm_greedy takes bf16 activations and packed bf16 weights")
        if workspace.numel() * workspace.element_size() < lm_greedy_workspace_bytes(M, N):
            raise ValueError("kw_dec_lm_greedy workspace too small")
        ldx = K if ldx is None else ldx
        self.tag = tag
        a = L.DecLinearArgs()
        a.x, a.ldx, a.ln, a.ln_eps, a.ln_colsum = x.data_ptr() + x_offset * 2, ldx, 1, float(eps), colsum.data_ptr()
        a.W, a.bias = W.data_ptr(), bias.data_ptr() if bias is not None else None
        a.epilogue, a.C, a.ldc, a.c_dtype = L.KW_EPI_STORE, _p(logits), logits.stride(0) if logits is not None else N, L.KW_DT_F32
        a.scale, a.M, a.N, a.K = 1.0, M, N, K
        g = L.SamplerArgs()
        g.B, g.V = M, N
        g.suppress_mask = suppress_mask.data_ptr()
        g.begin_suppress = begin_suppress.data_ptr() if begin_suppress is not None else None
        g.n_begin_suppress = begin_suppress.numel() if begin_suppress is not None else 0
        g.eos_id, g.pad_id, g.max_length, g.begin_index, g.max_initial_ts = eos_id, pad_id, max_length, begin_index, -1
        g.ids, g.ids_stride, g.cur_len = ids.data_ptr(), ids.stride(0), cur_len.data_ptr()
        g.unfinished, g.n_unfinished = unfinished.data_ptr(), n_unfinished.data_ptr()
        g.workspace, g.ws_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
        self._a, self._g = a, g
        self._ra, self._rg = ctypes.byref(a), ctypes.byref(g)
        self._keep = (x, W, bias, colsum, logits, suppress_mask, begin_suppress, ids, cur_len, unfinished, n_unfinished,
                      workspace)
        self._targs = (x, W, bias, colsum, logits, suppress_mask, begin_suppress, ids, cur_len, unfinished, n_unfinished,
                       workspace, [x_offset, ldx, M, N, K], float(eps), [eos_id, pad_id, max_length, begin_index])

    def __call__(self):
        if _BACKEND == "torch":
            _kw().dec_lm_greedy(*self._targs)
        else:
            L.check(_lib().kw_dec_lm_greedy(self._ra, self._rg, _s()), "kw_dec_lm_greedy")


class BeamStepPlan:
    """Pre-built ``kw_beam_logprobs`` + ``kw_beam_select`` calls for one beam-search step."""

    def __init__(self, st, logits, suppress_mask, begin_suppress, *, return_timestamps, ts_begin, no_ts_id, eos_id,
                 max_initial_ts, begin_index, max_length, fill_id, length_penalty, early_stopping):
        """``st``: a dict of the device state tensors (see DecodeSession.generate_beam)."""
        self._keep = (st, logits, suppress_mask, begin_suppress)
        R, V = logits.shape
        B, nb = st["fin_score"].shape
        mit = -1 if max_initial_ts is None else max_initial_ts
        es = 2 if early_stopping == "never" else int(bool(early_stopping))
        ws = st.get("lp_ws")  # split-row log-probs / top-k (kw_beam_logprobs_workspace), zero-filled once
        bp = st.get("bp")
        self._tlp = (logits, suppress_mask, begin_suppress, st["ids"], st["cur_len"], st["cand_val"], st["cand_idx"],
                     st["done"], ws, [int(bool(return_timestamps)), ts_begin, no_ts_id, eos_id, mit, begin_index, 2 * nb])
        self._tsel = (st["cand_val"], st["cand_idx"], st["ids"], bp, st["run_scores"], st["fin_seq"], st["fin_score"],
                      st["fin_len"], st["fin_flag"], st["unsat"], st["cur_len"], st["counter"], st["go"], st["done"],
                      st["item_flags"], [B, nb, V, begin_index, max_length, eos_id, fill_id, es], float(length_penalty))
        a = L.BeamLogprobsArgs()
        a.logits, a.R, a.V = logits.data_ptr(), R, V
        a.suppress_mask = suppress_mask.data_ptr()
        a.begin_suppress = begin_suppress.data_ptr() if begin_suppress is not None else None
        a.n_begin_suppress = begin_suppress.numel() if begin_suppress is not None else 0
        a.return_timestamps = int(bool(return_timestamps))
        a.ts_begin, a.no_ts_id, a.eos_id = ts_begin, no_ts_id, eos_id
        a.max_initial_ts = mit
        a.ids, a.ids_stride = st["ids"].data_ptr(), st["ids"].stride(0)
        a.cur_len = st["cur_len"].data_ptr()
        a.begin_index = begin_index
        a.k = 2 * nb
        a.cand_val, a.cand_idx, a.done = st["cand_val"].data_ptr(), st["cand_idx"].data_ptr(), st["done"].data_ptr()
        a.workspace = ws.data_ptr() if ws is not None else None
        a.ws_bytes = ws.numel() * ws.element_size() if ws is not None else 0
        b = L.BeamSelectArgs()
        b.B, b.num_beams, b.V = B, nb, V
        b.cand_val, b.cand_idx = a.cand_val, a.cand_idx
        b.ids, b.ids_stride = a.ids, a.ids_stride
        b.bp = bp.data_ptr() if bp is not None else None
        b.bp_stride = bp.stride(0) if bp is not None else 0
        b.run_scores = st["run_scores"].data_ptr()
        b.fin_seq, b.fin_stride = st["fin_seq"].data_ptr(), st["fin_seq"].shape[-1]
        b.fin_score, b.fin_len, b.fin_flag = st["fin_score"].data_ptr(), st["fin_len"].data_ptr(), st["fin_flag"].data_ptr()
        b.unsat, b.cur_len = st["unsat"].data_ptr(), a.cur_len
        b.begin_index, b.max_length, b.eos_id, b.fill_id = begin_index, max_length, eos_id, fill_id
        b.length_penalty = float(length_penalty)
        b.early_stopping = es
        b.counter, b.go, b.done = st["counter"].data_ptr(), st["go"].data_ptr(), a.done
        b.item_flags = st["item_flags"].data_ptr()
        self.a, self.b = a, b
        self._ra, self._rb = ctypes.byref(a), ctypes.byref(b)

    def __call__(self):
        if _BACKEND == "torch":
            kw = _kw()
            kw.beam_logprobs(*self._tlp)
            kw.beam_select(*self._tsel)
        else:
            L.check(_lib().kw_beam_logprobs(self._ra, _s()), "kw_beam_logprobs")
            L.check(_lib().kw_beam_select(self._rb, _s()), "kw_beam_select")
