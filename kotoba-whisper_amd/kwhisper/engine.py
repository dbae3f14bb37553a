"""WhisperEngine: weights in HBM, the encoder pass and device-resident decode sessions.

Mirrors the compute of ``WhisperForConditionalGeneration`` (TF/models/whisper/modeling_whisper.py):
encoder :592-646, decoder :690-795, proj_out :1080.  Every op is a kwhisper HIP kernel launched through
the ``torch.ops.kw`` custom ops over the C ABI; torch only owns memory, streams and graph capture.

Layout in HBM (DESIGN.md §Data layout):
  * encoder residual stream [rows][d]: bf16 on the bf16 path (the reference's bf16 model keeps it in
    bf16; the LayerNorm adds the producing linear's bf16 output into it), f32 in the parity mode;
    decoder residual f32 with a bf16 mirror; GEMM inputs (LayerNorm outputs) in the compute dtype;
  * conv stem: mel -> time-major zero-padded [B][3002][c_pad], conv1 output [B][3002][d]
    (pad rows stay zero), so both convolutions are im2col-free GEMMs;
  * encoder q/k/v head-split [3][B][H][1500][64]; the cross-attention K/V of all decoder layers from ONE
    GEMM straight into the static cache [2L][B][H][1500][64];
  * decoder self K/V static cache [L][B][H][448][64]; decode-step weights pre-packed into 1-KB MFMA
    fragments (bf16) for the skinny GEMMs.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib as L
from . import ops
from .config import GenerationConstants, WhisperShape, generation_constants

_HD = 64


def _to_tensor(v) -> torch.Tensor:
    if isinstance(v, torch.Tensor):
        return v.detach().float()
    return torch.from_numpy(np.asarray(v, dtype=np.float32))


class _EncoderBuffers:
    def __init__(self, eng: "WhisperEngine", B: int, out: torch.Tensor | None = None):
        s, dev, dt = eng.shape, eng.device, eng.dtype
        d, T = s.d_model, s.max_source_positions
        self.B = B
        self.mel_tm = torch.empty((B, s.n_frames + 2, eng.c_pad), device=dev, dtype=dt)
        self.conv = torch.zeros((B, s.n_frames + 2, d), device=dev, dtype=dt)  # pad rows stay zero
        # residual stream: f32 in the parity mode; bf16 on the bf16 path -- the reference model's own
        # residual precision (run_pseudo_labelling.py:229 loads the teacher in bfloat16)
        self.h = torch.empty((B * T, d), device=dev, dtype=torch.float32 if dt == torch.float32 else dt)
        self.x = torch.empty((B * T, d), device=dev, dtype=dt)
        self.qkv = torch.empty((3 * B * T * d,), device=dev, dtype=dt)
        self.attn = torch.empty((B * T, d), device=dev, dtype=dt)
        self.ffn = torch.empty((B * T, s.encoder_ffn_dim), device=dev, dtype=dt)
        self.out = torch.empty((B * T, d), device=dev, dtype=dt) if out is None else out
        # bf16 path: out-proj / fc2 store their output here and the next LayerNorm adds it into h
        # (a bf16 store is cheaper than the f32 read-modify-write of a residual epilogue)
        self.delta = torch.empty((B * T, d), device=dev, dtype=dt) if dt == torch.bfloat16 else None
        self.plans = eng._encoder_plans(self)


class WhisperEngine:
    """The MI355X Whisper model: ``encode`` (mel -> hidden) and decode sessions.

    ``dtype`` = torch.bfloat16 (performance path, bf16 MFMA with f32 accumulation) or
    torch.float32 (parity path: exact-fp32 MFMA; greedy tokens match the fp32 reference).
    """

    def __init__(self, shape: WhisperShape, state_dict: dict, *, dtype=torch.bfloat16, device="cuda",
                 generation_config: GenerationConstants | None = None, fuse_qkv_self: bool = True,
                 fuse_xq_cross: bool = True, encoder_streams: int = 2, prefill_streams: int = 2,
                 steps_per_replay: int = 2, fuse_lm_greedy: bool = True):
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("dtype must be torch.bfloat16 or torch.float32")
        L.load()
        L.load_torch_ops()  # torch.ops.kw.* (the launch path of every op); raises if it was not built
        self.shape = shape
        self.dtype = dtype
        # greedy bf16 decode steps run each layer's QKV projection + self-attention as one kw_dec_qkv_self launch
        # (caches bitwise the two-launch plan's, attention within bf16 rounding; False keeps the two launches)
        self.fuse_qkv_self = bool(fuse_qkv_self)
        # ... and each layer's cross-attention query projection + cross-attention step as one kw_dec_xq_cross launch
        # (bitwise the two-launch plan; False keeps the two launches)
        self.fuse_xq_cross = bool(fuse_xq_cross)
        # (fc1 -> fc2 stays two launches: both fused designs lost -- r04's 19.8 and r05's co-resident 22.4-23.3 vs
        # 18.4-18.6 us; the lab keeps them, tools/lab/mlp_coresident.py, profiles/r05b_mlp_decomposition.txt)
        # the encoder's batch as this many parts, their kernels issued interleaved on as many side streams: each
        # GEMM's last round of 256-row tiles leaves CUs idle that the other part's kernels fill (rows are
        # independent, so the output is bitwise the one-pass encoder's; large-v3 B = 32: 70.5 -> 67.6 ms,
        # profiles/r03_lab_notes.md r03ag)
        self.encoder_streams = max(1, int(encoder_streams))
        # ... and the greedy prefill (the prompt's pass) as this many row views of the session on side streams
        # (DecodeSession._run_prefill; tokens identical; 5.65 -> 5.2 ms at large-v3 B = 32, r03ah)
        self.prefill_streams = max(1, int(prefill_streams))
        # greedy decode steps per hipGraph replay (DecodeSession.generate: one launch, one unfinished-count copy and
        # event per replay; the host's stop check keeps the same lag in steps)
        self.steps_per_replay = max(1, int(steps_per_replay))
        # greedy bf16 decode steps without timestamps run the LM head and the greedy step as one kw_dec_lm_greedy
        # launch (the same tokens; False keeps kw_dec_linear + kw_greedy_step)
        self.fuse_lm_greedy = bool(fuse_lm_greedy)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("WhisperEngine runs on a cuda (HIP) device only")
        self.generation_config = generation_config or generation_constants(shape)
        d = shape.d_model
        self.H = shape.encoder_attention_heads
        if d // self.H != _HD:
            raise ValueError("head_dim must be 64")
        self.c_pad = (-(-shape.num_mel_bins // 64) * 64) if dtype == torch.bfloat16 else (-(-shape.num_mel_bins // 16) * 16)
        self._load(state_dict)
        self._enc = {}
        self._enc_split = {}
        self._enc_streams = []

    # ------------------------------------------------------------------------------------------
    def _dev(self, t: torch.Tensor, dtype=None) -> torch.Tensor:
        return t.to(device=self.device, dtype=dtype or self.dtype).contiguous()

    def _load(self, sd: dict) -> None:
        s = self.shape
        d = s.d_model
        g = lambda n: _to_tensor(sd[n])  # noqa: E731
        f32 = torch.float32
        # conv stem as GEMMs: W'[o][k*C + c] = W[o][c][k]
        w1 = g("model.encoder.conv1.weight")  # (d, n_mels, 3)
        w1p = torch.zeros((d, 3, self.c_pad), device=w1.device)
        w1p[:, :, : s.num_mel_bins] = w1.permute(0, 2, 1)
        self.conv1_w = self._dev(w1p.reshape(d, 3 * self.c_pad))
        self.conv1_b = self._dev(g("model.encoder.conv1.bias"), f32)
        self.conv2_w = self._dev(g("model.encoder.conv2.weight").permute(0, 2, 1).reshape(d, 3 * d))
        self.conv2_b = self._dev(g("model.encoder.conv2.bias"), f32)
        self.enc_pos = self._dev(g("model.encoder.embed_positions.weight"), f32)
        zero = torch.zeros(d, device=w1.device)

        def attn_qkv(p):
            w = torch.cat([g(f"{p}.q_proj.weight"), g(f"{p}.k_proj.weight"), g(f"{p}.v_proj.weight")], 0)
            b = torch.cat([g(f"{p}.q_proj.bias"), zero, g(f"{p}.v_proj.bias")], 0)
            return w, b

        self.enc_layers = []
        for i in range(s.encoder_layers):
            p = f"model.encoder.layers.{i}"
            qkv_w, qkv_b = attn_qkv(f"{p}.self_attn")
            self.enc_layers.append(dict(
                ln1_g=self._dev(g(f"{p}.self_attn_layer_norm.weight"), f32),
                ln1_b=self._dev(g(f"{p}.self_attn_layer_norm.bias"), f32),
                qkv_w=self._dev(qkv_w), qkv_b=self._dev(qkv_b, f32),
                o_w=self._dev(g(f"{p}.self_attn.out_proj.weight")), o_b=self._dev(g(f"{p}.self_attn.out_proj.bias"), f32),
                ln2_g=self._dev(g(f"{p}.final_layer_norm.weight"), f32),
                ln2_b=self._dev(g(f"{p}.final_layer_norm.bias"), f32),
                fc1_w=self._dev(g(f"{p}.fc1.weight")), fc1_b=self._dev(g(f"{p}.fc1.bias"), f32),
                fc2_w=self._dev(g(f"{p}.fc2.weight")), fc2_b=self._dev(g(f"{p}.fc2.bias"), f32),
            ))
        self.enc_ln_g = self._dev(g("model.encoder.layer_norm.weight"), f32)
        self.enc_ln_b = self._dev(g("model.encoder.layer_norm.bias"), f32)

        # decoder
        self.tok_emb = self._dev(g("model.decoder.embed_tokens.weight"))
        self.dec_pos = self._dev(g("model.decoder.embed_positions.weight"))
        packed = self.dtype == torch.bfloat16
        self.packed = packed
        pk = ops.pack_weight if packed else (lambda w: w)
        self.dec_layers = []
        ckv_w, ckv_b = [], []
        def fold(w, b, ln):
            """Packed (bf16) path: the LayerNorm feeding this projection is fused into kw_dec_linear, which forms
            only (h - mean) * rstd; gamma/beta are folded here: W' = W diag(gamma), b' = b + W beta."""
            if not packed:
                return pk(self._dev(w)), self._dev(b, f32), None
            gam, bet = g(f"{ln}.weight").float(), g(f"{ln}.bias").float()
            w32 = w.float()
            wf = self._dev(w32 * gam[None, :])
            return pk(wf), self._dev(b.float() + w32 @ bet, f32), ops.ln_colsum(wf)

        for i in range(s.decoder_layers):
            p = f"model.decoder.layers.{i}"
            qkv_w, qkv_b, qkv_cs = fold(*attn_qkv(f"{p}.self_attn"), f"{p}.self_attn_layer_norm")
            xq_w, xq_b, xq_cs = fold(g(f"{p}.encoder_attn.q_proj.weight"), g(f"{p}.encoder_attn.q_proj.bias"),
                                     f"{p}.encoder_attn_layer_norm")
            fc1_w, fc1_b, fc1_cs = fold(g(f"{p}.fc1.weight"), g(f"{p}.fc1.bias"), f"{p}.final_layer_norm")
            lay = dict(
                ln1_g=self._dev(g(f"{p}.self_attn_layer_norm.weight"), f32),
                ln1_b=self._dev(g(f"{p}.self_attn_layer_norm.bias"), f32),
                qkv_w=qkv_w, qkv_b=qkv_b, qkv_cs=qkv_cs,
                o_w=pk(self._dev(g(f"{p}.self_attn.out_proj.weight"))),
                o_b=self._dev(g(f"{p}.self_attn.out_proj.bias"), f32),
                ln2_g=self._dev(g(f"{p}.encoder_attn_layer_norm.weight"), f32),
                ln2_b=self._dev(g(f"{p}.encoder_attn_layer_norm.bias"), f32),
                xq_w=xq_w, xq_b=xq_b, xq_cs=xq_cs,
                xo_w=pk(self._dev(g(f"{p}.encoder_attn.out_proj.weight"))),
                xo_b=self._dev(g(f"{p}.encoder_attn.out_proj.bias"), f32),
                ln3_g=self._dev(g(f"{p}.final_layer_norm.weight"), f32),
                ln3_b=self._dev(g(f"{p}.final_layer_norm.bias"), f32),
                fc1_w=fc1_w, fc1_b=fc1_b, fc1_cs=fc1_cs,
                fc2_w=pk(self._dev(g(f"{p}.fc2.weight"))), fc2_b=self._dev(g(f"{p}.fc2.bias"), f32),
            )
            self.dec_layers.append(lay)
            ckv_w += [g(f"{p}.encoder_attn.k_proj.weight"), g(f"{p}.encoder_attn.v_proj.weight")]
            ckv_b += [zero, g(f"{p}.encoder_attn.v_proj.bias")]
        self.cross_kv_w = self._dev(torch.cat(ckv_w, 0))
        self.cross_kv_b = self._dev(torch.cat(ckv_b, 0), f32)
        self.dec_ln_g = self._dev(g("model.decoder.layer_norm.weight"), f32)
        self.dec_ln_b = self._dev(g("model.decoder.layer_norm.bias"), f32)
        if packed:  # final LayerNorm folded into the packed LM head (kw_dec_linear forms only (x-mean)*rstd)
            lg, lb = g("model.decoder.layer_norm.weight").float(), g("model.decoder.layer_norm.bias").float()
            e32 = g("model.decoder.embed_tokens.weight").float()
            lwf = self._dev(e32 * lg[None, :])
            self.lm_w, self.lm_cs = pk(lwf), ops.ln_colsum(lwf)
            self.lm_b = self._dev(e32 @ lb, f32)
            del lwf
            del e32
        else:
            self.lm_w, self.lm_b, self.lm_cs = self.tok_emb, None, None
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------------------------------
    # encoder
    # ------------------------------------------------------------------------------------------
    def _encoder_plans(self, bf: _EncoderBuffers):
        s, B, d = self.shape, bf.B, self.shape.d_model
        T, F = s.max_source_positions, s.n_frames
        M = B * T
        eps = s.layer_norm_eps
        plans = []
        plans.append(ops.GemmPlan(bf.mel_tm, self.conv1_w, bf.conv, B * F, d, 3 * self.c_pad, bias=self.conv1_b,
                                  lda=self.c_pad, a_rows_per_batch=F, a_batch_stride=(F + 2) * self.c_pad,
                                  ldc=d, c_rows_per_batch=F, c_batch_stride=(F + 2) * d, c_offset=d, gelu=True))
        plans.append(ops.GemmPlan(bf.conv, self.conv2_w, bf.h, M, d, 3 * d, bias=self.conv2_b,
                                  lda=2 * d, a_rows_per_batch=T, a_batch_stride=(F + 2) * d,
                                  gelu=True, row_add=self.enc_pos, row_add_period=T))
        # bf16: q also carries log2(e) (folded into the QKV epilogue's q scale: one bf16 rounding, as before), so
        # the attention's softmax takes its exponents straight off the matrix cores (kw_attention KW_ATTN_Q_LOG2)
        ql2 = self.dtype == torch.bfloat16
        scale = _HD ** -0.5 * (1.4426950408889634 if ql2 else 1.0)
        dl, pending = bf.delta, None  # pending: the delta the next LayerNorm must add into h first
        for lay in self.enc_layers:
            plans.append(("ln", bf.h, lay["ln1_g"], lay["ln1_b"], bf.x, pending))
            plans.append(ops.GemmPlan(bf.x, lay["qkv_w"], bf.qkv, M, 3 * d, d, bias=lay["qkv_b"],
                                      epilogue=L.KW_EPI_HEADSPLIT, scale=scale, scale_cols=d,
                                      hs_seq=T, hs_heads=self.H, hs_head_dim=_HD))
            plans.append(("attn", bf.qkv, bf.attn, ql2))
            if dl is None:
                plans.append(ops.GemmPlan(bf.attn, lay["o_w"], bf.h, M, d, d, bias=lay["o_b"], epilogue=L.KW_EPI_RESID))
            else:
                plans.append(ops.GemmPlan(bf.attn, lay["o_w"], dl, M, d, d, bias=lay["o_b"]))
            plans.append(("ln", bf.h, lay["ln2_g"], lay["ln2_b"], bf.x, dl))
            plans.append(ops.GemmPlan(bf.x, lay["fc1_w"], bf.ffn, M, s.encoder_ffn_dim, d, bias=lay["fc1_b"], gelu=True))
            if dl is None:
                plans.append(ops.GemmPlan(bf.ffn, lay["fc2_w"], bf.h, M, d, s.encoder_ffn_dim, bias=lay["fc2_b"],
                                          epilogue=L.KW_EPI_RESID))
            else:
                plans.append(ops.GemmPlan(bf.ffn, lay["fc2_w"], dl, M, d, s.encoder_ffn_dim, bias=lay["fc2_b"]))
            pending = dl
        plans.append(("ln", bf.h, self.enc_ln_g, self.enc_ln_b, bf.out, pending))
        return plans

    def encoder_buffers(self, B: int) -> _EncoderBuffers:
        if B not in self._enc:
            self._enc[B] = _EncoderBuffers(self, B)
        return self._enc[B]

    def encode(self, mel: torch.Tensor) -> torch.Tensor:
        """mel (B, n_mels, 3000) -> encoder last_hidden_state as (B*1500, d) in the compute dtype.

        Mirrors WhisperEncoder.forward (modeling_whisper.py:592-646), including its frame check.
        """
        s = self.shape
        if mel.dim() != 3 or mel.shape[1] != s.num_mel_bins:
            raise ValueError(f"input_features must be (batch, {s.num_mel_bins}, frames)")
        if mel.shape[-1] != s.n_frames:
            raise ValueError(
                f"Whisper expects the mel input features to be of length {s.n_frames}, but found {mel.shape[-1]}. "
                f"Make sure to pad the input mel features to {s.n_frames}."
            )
        mel = mel.to(device=self.device, dtype=torch.float32).contiguous()
        B = mel.shape[0]
        parts = min(self.encoder_streams, B)
        if parts > 1:
            return self._encode_split(mel, parts)
        bf = self.encoder_buffers(B)
        ops.mel_to_time_major(mel, self.c_pad, self.dtype, out=bf.mel_tm)
        for p in bf.plans:
            self._enc_op(p, B)
        return bf.out

    def _enc_op(self, p, B: int) -> None:
        if isinstance(p, tuple):
            if p[0] == "ln":
                ops.layernorm(p[1], p[2], p[3], self.shape.layer_norm_eps, p[4], delta=p[5])
            else:
                ops.attention(p[1], B, self.H, self.shape.max_source_positions, _HD, p[2], q_log2=p[3])
        else:
            p()

    def _encode_split(self, mel: torch.Tensor, parts: int) -> torch.Tensor:
        """encode() over ``parts`` row blocks of the batch, each with its own buffers and side stream, their
        launches issued in lockstep (plan i of every part, then plan i + 1) so that one part's kernels run in
        the CUs another part's kernel leaves idle.  Each part writes its rows of one (B*T, d) output."""
        s, B = self.shape, mel.shape[0]
        T, d = s.max_source_positions, s.d_model
        sizes = [B // parts + (1 if i < B % parts else 0) for i in range(parts)]
        key = (B, tuple(sizes))
        if key not in self._enc_split:
            out = torch.empty((B * T, d), device=self.device, dtype=self.dtype)
            bufs, r0 = [], 0
            for n in sizes:
                bufs.append(_EncoderBuffers(self, n, out=out[r0 * T:(r0 + n) * T]))
                r0 += n
            self._enc_split[key] = (out, bufs)
        out, bufs = self._enc_split[key]
        while len(self._enc_streams) < parts:
            self._enc_streams.append(L.new_stream(self.device, owner=self))
        streams = self._enc_streams[:parts]
        cur = torch.cuda.current_stream(self.device)
        r0 = 0
        for bf, st, n in zip(bufs, streams, sizes):
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                ops.mel_to_time_major(mel[r0:r0 + n], self.c_pad, self.dtype, out=bf.mel_tm)
            r0 += n
        for j in range(len(bufs[0].plans)):
            for bf, st in zip(bufs, streams):
                with torch.cuda.stream(st):
                    self._enc_op(bf.plans[j], bf.B)
        for st in streams:  # (the join also orders any later reuse of mel's memory after the parts' reads)
            cur.wait_stream(st)
        return out

    # ------------------------------------------------------------------------------------------
    def cross_kv(self, enc: torch.Tensor, B: int, out: torch.Tensor | None = None) -> torch.Tensor:
        """All decoder layers' cross-attention K/V in one GEMM: [2L][B][H][1500][64] (modeling_whisper.py:323-335)."""
        s = self.shape
        T, d = s.max_source_positions, s.d_model
        n = 2 * s.decoder_layers * d
        if out is None:
            out = torch.empty((2 * s.decoder_layers, B, self.H, T, _HD), device=self.device, dtype=self.dtype)
        ops.GemmPlan(enc, self.cross_kv_w, out, B * T, n, d, bias=self.cross_kv_b, epilogue=L.KW_EPI_HEADSPLIT,
                     hs_seq=T, hs_heads=self.H, hs_head_dim=_HD)()
        return out

    def lane(self) -> "WhisperEngine":
        """Another handle on this engine's weights with its own activation buffers and side streams, so a second
        host thread can run batches at the same time as this one (each thread on its own current stream, each
        with its own KWhisperForConditionalGeneration and decode sessions).  Nothing is copied on the device."""
        import copy

        other = copy.copy(self)
        other._enc, other._enc_split, other._enc_streams = {}, {}, []
        return other

    def new_session(self, B: int, enc: torch.Tensor | None = None, beams: int = 1) -> "DecodeSession":
        from .decode import CAPTURE_LOCK, DecodeSession

        with CAPTURE_LOCK:  # allocations must not interleave with another lane's capture
            return DecodeSession(self, B, enc, beams=beams)
