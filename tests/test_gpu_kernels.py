"""Kernel-level parity on the MI355X: every C-ABI entry point against the oracle / an fp32 reference.

Floating-point tolerances are stated per test.  Integer / index outputs (tokens, argmax, ids) are
compared exactly.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from kwhisper import _lib as L  # noqa: E402
from kwhisper import ops  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L.load()
    torch.manual_seed(0)


def dev(x, dtype=None):
    t = torch.as_tensor(x)
    return t.to("cuda", dtype or t.dtype).contiguous()


# ---------------------------------------------------------------- log-mel (a1)
@pytest.mark.parametrize("n_mels", [80, 128])
def test_log_mel_vs_oracle(n_mels):
    from oracle.mel import log_mel, mel_filters, pad_or_trim
    from kwhisper import synthetic as S
    from kwhisper.feature_extraction import mel_filter_bank

    clips = [S.dummy_audio(0), S.dummy_audio(1), S.tone_audio(0), S.tone_audio(1),
             pad_or_trim(S.tone_audio(2)[:24000]), np.zeros(480000, np.float32)]
    audio = np.stack(clips)
    fb = mel_filter_bank(201, n_mels, 0.0, 8000.0, 16000)
    np.testing.assert_allclose(fb, mel_filters(n_mels), rtol=1e-12, atol=1e-15)  # product bank == oracle bank
    got = ops.log_mel(dev(audio), dev(fb.astype(np.float32))).cpu().numpy()
    want = log_mel(audio, n_mels)
    err = np.abs(got - want).max()
    print("log-mel max abs err", err)
    # reference's own numpy-vs-torch tolerance is 1e-5 (feature_extraction_whisper.py:107)
    assert err < 2e-5


def test_log_mel_rejects_bad_length():
    with pytest.raises(ValueError):
        ops.log_mel(torch.zeros((1, 1000), device="cuda"), torch.zeros((201, 80), device="cuda"))


# ---------------------------------------------------------------- GEMMs
def _ref_gemm(A, W, bias):
    return A.float() @ W.float().t() + (bias if bias is not None else 0)


@pytest.mark.parametrize("M,N,K", [(256, 128, 64), (6000, 1152, 384), (1000, 384, 1536), (48000, 1280, 1280)])
def test_gemm_bf16_store(M, N, K):
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.GemmPlan(A, W, C, M, N, K, bias=b)()
    ref = _ref_gemm(A, W, b)
    torch.testing.assert_close(C.float(), ref, atol=2e-2, rtol=1e-2)


def test_gemm_bf16_epilogues():
    M, N, K = 300, 256, 128
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    ref = _ref_gemm(A, W, b)
    # gelu + column scale + row_add (period 7) into f32
    ra = torch.randn(7, N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    ops.GemmPlan(A, W, C, M, N, K, bias=b, gelu=True, scale=0.125, scale_cols=100, row_add=ra, row_add_period=7)()
    r = torch.nn.functional.gelu(ref)
    r[:, :100] *= 0.125
    r += ra[torch.arange(M, device="cuda") % 7]
    torch.testing.assert_close(C, r, atol=1e-3, rtol=1e-3)
    # residual add
    H0 = torch.randn(M, N, device="cuda")
    Hc = H0.clone()
    ops.GemmPlan(A, W, Hc, M, N, K, bias=b, epilogue=L.KW_EPI_RESID)()
    torch.testing.assert_close(Hc, H0 + ref, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("M,K", [(2000, 64), (2000, 128), (1100, 320), (4096, 1280)])
def test_gemm256_pipeline_and_epilogues(M, K):
    """The 256x256 ping-pong kernel (N % 256 == 0, M >= 1024): K-tile counts 1, 2, odd, 20; ragged last
    row tile; STORE (gelu + column scale + row_add) and RESID epilogues."""
    N = 512
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    ref = _ref_gemm(A, W, b)
    ra = torch.randn(5, N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    ops.GemmPlan(A, W, C, M, N, K, bias=b, gelu=True, scale=0.125, scale_cols=300, row_add=ra, row_add_period=5)()
    r = torch.nn.functional.gelu(ref)
    r[:, :300] *= 0.125
    r += ra[torch.arange(M, device="cuda") % 5]
    torch.testing.assert_close(C, r, atol=1e-3, rtol=1e-3)
    H0 = torch.randn(M, N, device="cuda")
    Hc = H0.clone()
    ops.GemmPlan(A, W, Hc, M, N, K, bias=b, epilogue=L.KW_EPI_RESID)()
    torch.testing.assert_close(Hc, H0 + ref, atol=1e-3, rtol=1e-3)
    Cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.GemmPlan(A, W, Cb, M, N, K, bias=b)()
    torch.testing.assert_close(Cb.float(), ref, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("M,K,bias", [(33000, 64, True), (33000, 192, False), (70001, 128, True)])
def test_gemm256_persistent(M, K, bias):
    """More tiles than CUs: each persistent workgroup walks several tiles, the next tile's prologue
    overlapping this one's epilogue (STORE bf16/f32); RESID and row_add take the serial hand-off."""
    N = 1024
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda") if bias else None
    ref = _ref_gemm(A, W, b)
    Cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.GemmPlan(A, W, Cb, M, N, K, bias=b, gelu=True, scale=0.5, scale_cols=200)()
    r = torch.nn.functional.gelu(ref)
    r[:, :200] *= 0.5
    torch.testing.assert_close(Cb.float(), r, atol=2e-2, rtol=1e-2)
    C = torch.empty(M, N, device="cuda")
    ops.GemmPlan(A, W, C, M, N, K, bias=b)()
    torch.testing.assert_close(C, ref, atol=1e-3, rtol=1e-3)
    ra = torch.randn(7, N, device="cuda")
    ops.GemmPlan(A, W, C, M, N, K, bias=b, row_add=ra, row_add_period=7)()
    torch.testing.assert_close(C, ref + ra[torch.arange(M, device="cuda") % 7], atol=1e-3, rtol=1e-3)
    ops.GemmPlan(A, W, Cb, M, N, K, bias=b, row_add=ra, row_add_period=7)()  # bf16 + row_add (the conv2 stem)
    torch.testing.assert_close(Cb.float(), ref + ra[torch.arange(M, device="cuda") % 7], atol=2e-2, rtol=1e-2)
    H0 = torch.randn(M, N, device="cuda")
    Hc = H0.clone()
    ops.GemmPlan(A, W, Hc, M, N, K, bias=b, epilogue=L.KW_EPI_RESID)()
    torch.testing.assert_close(Hc, H0 + ref, atol=1e-3, rtol=1e-3)


def test_gemm256_headsplit():
    B, T, H, hd = 24, 1500, 4, 64  # 141 x 3 tiles: persistent walk with the head-split store
    d = H * hd
    M, N, K = B * T, 3 * d, 256
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    C = torch.empty(3, B, H, T, hd, device="cuda", dtype=torch.bfloat16)
    ops.GemmPlan(A, W, C, M, N, K, bias=b, epilogue=L.KW_EPI_HEADSPLIT, scale=0.125, scale_cols=d,
                 hs_seq=T, hs_heads=H, hs_head_dim=hd)()
    ref = _ref_gemm(A, W, b)
    ref[:, :d] *= 0.125
    ref = ref.view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    torch.testing.assert_close(C.float(), ref, atol=2e-2, rtol=1e-2)


def test_gemm_bf16_headsplit():
    B, T, H, hd = 2, 100, 2, 64
    d = H * hd
    M, N, K = B * T, 3 * d, 128
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    C = torch.empty(3, B, H, T, hd, device="cuda", dtype=torch.bfloat16)
    ops.GemmPlan(A, W, C, M, N, K, bias=b, epilogue=L.KW_EPI_HEADSPLIT, scale=0.125, scale_cols=d,
                 hs_seq=T, hs_heads=H, hs_head_dim=hd)()
    ref = _ref_gemm(A, W, b)
    ref[:, :d] *= 0.125
    ref = ref.view(B, T, 3, H, hd).permute(2, 0, 3, 1, 4)
    torch.testing.assert_close(C.float(), ref, atol=2e-2, rtol=1e-2)


def test_gemm_conv_rowmap():
    """Conv1d(k3, p1, stride 1 and 2) as GEMM over the time-major padded layout."""
    B, C, T, d = 2, 80, 3000, 256
    mel = torch.randn(B, C, T, device="cuda")
    w1 = torch.randn(d, C, 3, device="cuda") / (3 * C) ** 0.5
    b1 = torch.randn(d, device="cuda")
    w2 = torch.randn(d, d, 3, device="cuda") / (3 * d) ** 0.5
    b2 = torch.randn(d, device="cuda")
    c_pad = 128
    tm = ops.mel_to_time_major(mel, c_pad, torch.bfloat16)
    w1p = torch.zeros(d, 3, c_pad, device="cuda")
    w1p[:, :, :C] = w1.permute(0, 2, 1)
    w1p = w1p.reshape(d, 3 * c_pad).bfloat16().contiguous()
    conv = torch.zeros(B, T + 2, d, device="cuda", dtype=torch.bfloat16)
    ops.GemmPlan(tm, w1p, conv, B * T, d, 3 * c_pad, bias=b1, lda=c_pad, a_rows_per_batch=T,
                 a_batch_stride=(T + 2) * c_pad, ldc=d, c_rows_per_batch=T, c_batch_stride=(T + 2) * d, c_offset=d,
                 gelu=True)()
    ref1 = torch.nn.functional.gelu(torch.nn.functional.conv1d(mel.bfloat16().float(), w1.bfloat16().float(), b1, padding=1))
    torch.testing.assert_close(conv[:, 1:-1].float().permute(0, 2, 1), ref1, atol=3e-2, rtol=2e-2)
    assert conv[:, 0].abs().max() == 0 and conv[:, -1].abs().max() == 0
    w2p = w2.permute(0, 2, 1).reshape(d, 3 * d).bfloat16().contiguous()
    Tn = T // 2
    pos = torch.randn(Tn, d, device="cuda")
    h = torch.empty(B * Tn, d, device="cuda")
    ops.GemmPlan(conv, w2p, h, B * Tn, d, 3 * d, bias=b2, lda=2 * d, a_rows_per_batch=Tn,
                 a_batch_stride=(T + 2) * d, gelu=True, row_add=pos, row_add_period=Tn)()
    ref2 = torch.nn.functional.gelu(torch.nn.functional.conv1d(conv[:, 1:-1].float().permute(0, 2, 1),
                                                                w2.bfloat16().float(), b2, stride=2, padding=1))
    ref2 = ref2.permute(0, 2, 1) + pos
    torch.testing.assert_close(h.view(B, Tn, d), ref2, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,N,K", [(37, 100, 48), (512, 1280, 1280), (4, 51865, 384)])
def test_gemm_f32_exactish(M, N, K):
    A = torch.randn(M, K, device="cuda")
    W = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    C = torch.empty(M, N, device="cuda")
    ops.GemmPlan(A, W, C, M, N, K, bias=b)()
    ref = (A.double() @ W.double().t() + b.double()).float()
    torch.testing.assert_close(C, ref, atol=2e-5, rtol=2e-5)


@pytest.mark.parametrize("M,N,K", [(1, 1280, 1280), (32, 3840, 1280), (32, 1280, 5120), (128, 5120, 1280),
                                   (5, 51866, 1280), (32, 51865, 384), (17, 1152, 384), (32, 384, 1536)])
def test_dec_linear_store(M, N, K):
    """Plain decode linear (bf16 x, packed W, f32 and bf16 C) against an fp32 reference of the same op."""
    A = torch.randn(M, K, device="cuda").bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    Wp = ops.pack_weight(W)
    C = torch.empty(M, N, device="cuda")
    ops.DecLinearPlan(A, Wp, M, N, K, bias=b, C=C)()
    ref = _ref_gemm(A, W, b)
    torch.testing.assert_close(C, ref, atol=2e-3, rtol=2e-3)
    Cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.DecLinearPlan(A, Wp, M, N, K, bias=b, C=Cb, gelu=True, scale=0.5, scale_cols=N // 3)()
    r = torch.nn.functional.gelu(ref)
    r[:, : N // 3] *= 0.5
    torch.testing.assert_close(Cb.float(), r, atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("rows,dim", [(1, 384), (48000, 1280), (33, 2048)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_layernorm(rows, dim, out_dtype):
    x = torch.randn(rows, dim, device="cuda") * 3 + 1
    g = torch.randn(dim, device="cuda")
    b = torch.randn(dim, device="cuda")
    y = torch.empty(rows, dim, device="cuda", dtype=out_dtype)
    ops.layernorm(x, g, b, 1e-5, y)
    ref = torch.nn.functional.layer_norm(x.double(), (dim,), g.double(), b.double(), 1e-5).float()
    tol = 1e-5 if out_dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), ref, atol=tol * 4, rtol=tol)


@pytest.mark.parametrize("rows,dim", [(3, 384), (48000, 1280), (5, 2048), (2, 8)])
@pytest.mark.parametrize("with_delta", [False, True])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_layernorm_bf16_residual(rows, dim, with_delta, out_dtype):
    """bf16 residual stream (encoder bf16 path): x = bf16(x + delta) written back bit-exactly, then the
    LayerNorm of the rounded sum (torch fp32/f64 references of the same op)."""
    x = (torch.randn(rows, dim, device="cuda") * 3 + 1).to(torch.bfloat16)
    delta = (torch.randn(rows, dim, device="cuda") * 2).to(torch.bfloat16) if with_delta else None
    g = torch.randn(dim, device="cuda")
    b = torch.randn(dim, device="cuda")
    want_h = (x.float() + delta.float()).to(torch.bfloat16) if with_delta else x.clone()
    y = torch.empty(rows, dim, device="cuda", dtype=out_dtype)
    ops.layernorm(x, g, b, 1e-5, y, delta=delta)
    assert torch.equal(x, want_h)
    ref = torch.nn.functional.layer_norm(want_h.double(), (dim,), g.double(), b.double(), 1e-5).float()
    tol = 1e-5 if out_dtype == torch.float32 else 2e-2
    torch.testing.assert_close(y.float(), ref, atol=tol * 4, rtol=tol)


@pytest.mark.parametrize("rows,dim", [(3, 384), (48000, 1280)])
def test_layernorm_residual_delta(rows, dim):
    """x += delta (bf16, written back) then LayerNorm: the encoder's fused residual add."""
    x = torch.randn(rows, dim, device="cuda") * 3 + 1
    delta = (torch.randn(rows, dim, device="cuda") * 2).to(torch.bfloat16)
    g = torch.randn(dim, device="cuda")
    b = torch.randn(dim, device="cuda")
    want_h = x + delta.float()
    y = torch.empty(rows, dim, device="cuda", dtype=torch.bfloat16)
    ops.layernorm(x, g, b, 1e-5, y, delta=delta)
    torch.testing.assert_close(x, want_h, atol=0, rtol=0)
    ref = torch.nn.functional.layer_norm(want_h.double(), (dim,), g.double(), b.double(), 1e-5).float()
    torch.testing.assert_close(y.float(), ref, atol=8e-2, rtol=2e-2)


# ---------------------------------------------------------------- attention
def _ref_attn(qkv, B, H, T, hd):
    q, k, v = qkv.float().view(3, B, H, T, hd)
    p = torch.softmax(q @ k.transpose(-1, -2), -1)
    return (p @ v).permute(0, 2, 1, 3).reshape(B, T, H * hd)


@pytest.mark.parametrize("B,H,T", [(1, 1, 64), (2, 3, 100), (2, 20, 1500), (1, 2, 1)])
def test_attention_bf16(B, H, T):
    hd = 64
    qkv = (torch.randn(3, B, H, T, hd, device="cuda") * 0.5).bfloat16()
    qkv[0] *= 0.125 * 8  # pre-scaled q of unit-ish size
    out = torch.empty(B, T, H * hd, device="cuda", dtype=torch.bfloat16)
    ops.attention(qkv, B, H, T, hd, out)
    torch.testing.assert_close(out.float(), _ref_attn(qkv, B, H, T, hd), atol=2e-2, rtol=2e-2)


def test_attention_bf16_spike():
    """Force the online-softmax rescale: one key dominates one query late in the sequence."""
    B, H, T, hd = 1, 1, 1500, 64
    qkv = (torch.randn(3, B, H, T, hd, device="cuda") * 0.3)
    qkv[1, 0, 0, 1400] = qkv[0, 0, 0, 5] * 40
    qkv = qkv.bfloat16()
    out = torch.empty(B, T, H * hd, device="cuda", dtype=torch.bfloat16)
    ops.attention(qkv, B, H, T, hd, out)
    torch.testing.assert_close(out.float(), _ref_attn(qkv, B, H, T, hd), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("B,H,T", [(2, 3, 100), (1, 4, 1500), (3, 2, 1501)])
def test_attention_bf16_q_log2(B, H, T):
    """KW_ATTN_Q_LOG2: q carries log2(e) (the bf16 engine's QKV epilogue folds it into the q scale) and the
    MFMA accumulates the scores onto -m_run, so p = exp2(s) is one v_exp per score.  Within bf16 rounding of
    fp32 softmax(q k^T) v for the q it was given (divided back by log2 e), as the natural-unit kernel is for
    its own, including a late dominant key (the reference moves) and a ragged last tile."""
    hd = 64
    qkv = (torch.randn(3, B, H, T, hd, device="cuda") * 0.5)
    qkv[0] *= 0.125 * 8
    qkv[1, 0, 0, T - 7] = qkv[0, 0, 0, 3] * 30  # one query's score spikes in the last tile
    q2 = qkv.clone()
    q2[0] *= 1.4426950408889634
    qkv, q2 = qkv.bfloat16(), q2.bfloat16()
    out = torch.empty(B, T, H * hd, device="cuda", dtype=torch.bfloat16)
    ops.attention(q2, B, H, T, hd, out, q_log2=True)
    ref_q = q2.float().clone()
    ref_q[0] /= 1.4426950408889634
    torch.testing.assert_close(out.float(), _ref_attn(ref_q, B, H, T, hd), atol=3e-2, rtol=2e-2)
    nat = torch.empty_like(out)  # the natural-unit kernel on its own (differently rounded) q: the same bar
    ops.attention(qkv, B, H, T, hd, nat)
    torch.testing.assert_close(nat.float(), _ref_attn(qkv, B, H, T, hd), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("B,H,T,ramp", [(2, 4, 1500, 40.0), (1, 3, 130, 60.0), (1, 2, 64, 20.0), (1, 2, 50, 0.0),
                                         (1, 2, 1, 0.0)])
def test_attention_bf16_q_log2_reference_moves(B, H, T, ramp):
    """attn_fwd_l2 computes p = exp2(s) before knowing whether the tile moves the exponent reference and redoes
    the tile only when some lane's row sum exceeds e^8: key scores that grow along the sequence make the
    reference move again and again (the rare branch in most tiles), a tile of <= 64 keys is both first and
    ragged, T = 1 has one key.  Within bf16 rounding of fp32 softmax(q k^T) v; the r03x lab run held it bitwise
    equal to the always-compute-the-maximum kernel it replaced (tools/lab/enc_attn_l2_ab.py)."""
    hd = 64
    g = torch.Generator(device="cuda").manual_seed(7)
    qkv = torch.randn(3, B, H, T, hd, device="cuda", generator=g) * 0.5
    qkv[0] *= 0.125 * 8 * 1.4426950408889634
    qkv[1] *= (1.0 + ramp * torch.arange(T, device="cuda", dtype=torch.float32) / T)[None, None, :, None]
    q2 = qkv.bfloat16()
    out = torch.full((B, T, H * hd), float("nan"), device="cuda", dtype=torch.bfloat16)
    ops.attention(q2, B, H, T, hd, out, q_log2=True)
    ref_q = q2.float().clone()
    ref_q[0] /= 1.4426950408889634
    ref = _ref_attn(ref_q, B, H, T, hd)
    assert torch.isfinite(out.float()).all()
    torch.testing.assert_close(out.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("B,H,T", [(2, 3, 100), (1, 6, 1500)])
def test_attention_f32(B, H, T):
    hd = 64
    qkv = torch.randn(3, B, H, T, hd, device="cuda") * 0.5
    out = torch.empty(B, T, H * hd, device="cuda")
    ops.attention(qkv, B, H, T, hd, out)
    ref = _ref_attn(qkv.double(), B, H, T, hd).float()
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("q_len,past", [(1, 10), (4, 10), (1, 255), (1, 256), (1, 300), (1, 447), (4, 300)])
def test_self_attn_step(dtype, q_len, past):
    """Cache append + attention; one new position splits at 256 keys (chunk combine), the prefill walks
    queries causally."""
    B, H, hd, t_max = 3, 4, 64, 448
    d = H * hd
    kc = torch.zeros(B, H, t_max, hd, device="cuda", dtype=dtype)
    vc = torch.zeros_like(kc)
    kc[:, :, :past] = torch.randn(B, H, past, hd, device="cuda").to(dtype)
    vc[:, :, :past] = torch.randn(B, H, past, hd, device="cuda").to(dtype)
    qkv = torch.randn(B * q_len, 3 * d, device="cuda").to(dtype)
    cur = torch.tensor([past + q_len], device="cuda", dtype=torch.int32)
    out = torch.empty(B * q_len, d, device="cuda", dtype=dtype)
    ws = torch.zeros(ops.self_attn_workspace_bytes(B, H, t_max) // 4 + 1, device="cuda")
    for _ in range(2):  # the arrival counters must come back to zero
        ops.self_attn_step(qkv, B, q_len, H, hd, kc, vc, t_max, cur, out, ws)
    x = qkv.float().view(B, q_len, 3, H, hd)
    k_all = torch.cat([kc[:, :, :past].float(), x[:, :, 1].permute(0, 2, 1, 3)], 2)
    v_all = torch.cat([vc[:, :, :past].float(), x[:, :, 2].permute(0, 2, 1, 3)], 2)
    q = x[:, :, 0].permute(0, 2, 1, 3)
    s = q @ k_all.transpose(-1, -2)
    mask = torch.arange(past + q_len, device="cuda")[None, :] > (torch.arange(q_len, device="cuda")[:, None] + past)
    s = s.masked_fill(mask, float("-inf"))
    ref = (torch.softmax(s, -1) @ v_all).permute(0, 2, 1, 3).reshape(B * q_len, d)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)
    torch.testing.assert_close(kc[:, :, past:past + q_len].float(), x[:, :, 1].permute(0, 2, 1, 3))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("q_len,S", [(1, 1500), (3, 1500), (1, 77), (1, 256), (1, 2048)])
def test_cross_attn_step(dtype, q_len, S):
    B, H, hd = 3, 4, 64
    d = H * hd
    k = torch.randn(B, H, S, hd, device="cuda").to(dtype)
    v = torch.randn(B, H, S, hd, device="cuda").to(dtype)
    q = (torch.randn(B * q_len, d, device="cuda") * 0.3).to(dtype)
    out = torch.empty(B * q_len, d, device="cuda", dtype=dtype)
    ws = torch.zeros(ops.cross_attn_workspace_bytes(B, q_len, H, hd, S) // 4 + 1, device="cuda")
    for _ in range(2):
        ops.cross_attn_step(q, B, q_len, H, hd, k, v, S, out, ws)
    qq = q.float().view(B, q_len, H, hd).permute(0, 2, 1, 3)
    ref = (torch.softmax(qq @ k.float().transpose(-1, -2), -1) @ v.float()).permute(0, 2, 1, 3).reshape(B * q_len, d)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(out.float(), ref, atol=tol, rtol=tol)
    _check_cross_ws_rearmed(ws, B * q_len * H, S)


def test_cross_attn_step_b32_repeated():
    """The bench shape (large-v3 B = 32, 20 heads, 1500 keys), 64 launches on one workspace: every launch equal
    (the granule combine is deterministic and re-arms itself), close to fp32, workspace left re-armed."""
    B, H, S, hd = 32, 20, 1500, 64
    torch.manual_seed(5)
    k = torch.randn(B, H, S, hd, device="cuda").bfloat16()
    v = torch.randn(B, H, S, hd, device="cuda").bfloat16()
    q = (torch.randn(B, H * hd, device="cuda") * 0.3).bfloat16()
    out = torch.empty(B, H * hd, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, hd, S) // 4 + 1, device="cuda")
    ops.cross_attn_step(q, B, 1, H, hd, k, v, S, out, ws)
    first = out.clone()
    for _ in range(63):
        ops.cross_attn_step(q, B, 1, H, hd, k, v, S, out, ws)
    assert torch.equal(out, first)
    qq = q.float().view(B, 1, H, hd).permute(0, 2, 1, 3)
    ref = (torch.softmax(qq @ k.float().transpose(-1, -2), -1) @ v.float()).permute(0, 2, 1, 3).reshape(B, H * hd)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    _check_cross_ws_rearmed(ws, B * H, S)


@pytest.mark.parametrize("B,H", [(32, 20), (13, 20), (44, 6)])
def test_cross_attn_step_pair_kernel(B, H):
    """One workgroup per (row, head) pair streaming its six 250-key chunks with the next chunk in flight
    (cross_attn_row_kernel: B H between the CU count and what fits at once -- 640, 260 and 264 pairs here):
    close to fp32 softmax(q K^T) V, deterministic, and it leaves the workspace untouched (zero)."""
    S, hd = 1500, 64
    torch.manual_seed(B * 100 + H)
    k = torch.randn(B, H, S, hd, device="cuda").bfloat16()
    v = torch.randn(B, H, S, hd, device="cuda").bfloat16()
    q = (torch.randn(B, H * hd, device="cuda") * 0.3).bfloat16()
    out = torch.empty(B, H * hd, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, hd, S) // 4 + 1, device="cuda")
    ops.cross_attn_step(q, B, 1, H, hd, k, v, S, out, ws)
    first = out.clone()
    for _ in range(3):
        ops.cross_attn_step(q, B, 1, H, hd, k, v, S, out, ws)
        assert torch.equal(out, first)
    qq = q.float().view(B, 1, H, hd).permute(0, 2, 1, 3)
    ref = (torch.softmax(qq @ k.float().transpose(-1, -2), -1) @ v.float()).permute(0, 2, 1, 3).reshape(B, H * hd)
    torch.testing.assert_close(out.float(), ref, atol=2e-2, rtol=2e-2)
    assert int(ws.view(torch.int32).abs().sum()) == 0


def test_cross_attn_batch_invariant():
    """A greedy row's cross-attention is bitwise the same whichever grid its batch size selects: B = 32 (640
    pairs: cross_attn_row_kernel, a wave folding its chunks as it streams) == the same rows in batches of 2
    (40 pairs: cross_attn_dma_kernel, per-wave chunk partials folded by the last chunk) -- also through the fused
    query projection (kw_dec_xq_cross: cross_attn_row_kernel<QG> vs xq_cross_kernel)."""
    B, H, S, hd = 32, 20, 1500, 64
    d = H * hd
    torch.manual_seed(11)
    k = torch.randn(B, H, S, hd, device="cuda").bfloat16()
    v = torch.randn(B, H, S, hd, device="cuda").bfloat16()
    q = (torch.randn(B, d, device="cuda") * 0.3).bfloat16()
    big = torch.empty(B, d, device="cuda", dtype=torch.bfloat16)
    ops.cross_attn_step(q, B, 1, H, hd, k, v, S, big, torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, hd, S) // 4 + 1,
                                                                   device="cuda"))
    ws2 = torch.zeros(ops.cross_attn_workspace_bytes(2, 1, H, hd, S) // 4 + 1, device="cuda")
    small = torch.empty(2, d, device="cuda", dtype=torch.bfloat16)
    for b0 in range(0, B, 2):
        ops.cross_attn_step(q[b0:b0 + 2].contiguous(), 2, 1, H, hd, k[b0:b0 + 2].contiguous(), v[b0:b0 + 2].contiguous(),
                            S, small, ws2)
        assert torch.equal(small, big[b0:b0 + 2]), b0
    _check_cross_ws_rearmed(ws2, 2 * H, S)
    # fused query projection
    eps = 1e-5
    hb = torch.randn(B, d, device="cuda").bfloat16()
    W = (torch.randn(d, d, device="cuda") / d ** 0.5).bfloat16()
    packed, colsum = ops.pack_weight(W), ops.ln_colsum(W)
    bias = torch.randn(d, device="cuda") * 0.1
    fb = torch.empty(B, d, device="cuda", dtype=torch.bfloat16)
    ops.XqCrossPlan(hb, packed, B, d, H, ln=(eps, colsum), bias=bias, scale=0.125, k=k, v=v, S=S, out=fb,
                    workspace=torch.zeros(ops.xq_cross_workspace_bytes(B, d, H, S) // 4 + 1, device="cuda"))()
    wsx = torch.zeros(ops.xq_cross_workspace_bytes(2, d, H, S) // 4 + 1, device="cuda")
    for b0 in range(0, B, 2):
        ops.XqCrossPlan(hb[b0:b0 + 2].contiguous(), packed, 2, d, H, ln=(eps, colsum), bias=bias, scale=0.125,
                        k=k[b0:b0 + 2].contiguous(), v=v[b0:b0 + 2].contiguous(), S=S, out=small, workspace=wsx)()
        assert torch.equal(small, fb[b0:b0 + 2]), b0
    torch.cuda.synchronize()
    assert int(wsx.view(torch.int32).abs().sum()) == 0


def _check_cross_ws_rearmed(ws, rows, S):
    """Every launch leaves the workspace as it needs the next one: arrival counters 0, the error word 0 (no
    granule poll timed out), every {value, tag} granule re-armed to 0 by its combining split."""
    ns = -(-S // 256)
    part = rows * ns * 66
    w = ws.view(torch.int32)
    assert int(w[part: part + rows].abs().sum()) == 0, "arrival counters not reset"
    assert int(w[part + rows]) == 0, "cross-attention granule poll timed out"
    g0 = (4 * (part + rows + 1) + 63) // 64 * 16  # granule region [rows][ns][4 waves][66] x 8 B, in int32 words
    assert int(w[g0: g0 + 8 * part].abs().sum()) == 0, "granules not re-armed"


@pytest.mark.parametrize("q_len", [2, 3, 4, 5, 8, 13, 20, 32, 45])
@pytest.mark.parametrize("S", [1500, 200])
def test_cross_attn_multirow_bitwise(q_len, S):
    """bf16 rows of one item sharing a K/V pass (prefill positions, beams) vs each row attended alone by
    the one-row kernel: up to 4 rows the same f32 arithmetic per chunk -- bit for bit with one chunk (S = 200);
    over several chunks the one-row kernels fold per-wave chunk partials (bitwise cross_attn_row_kernel's,
    so greedy rows are batch-invariant) while the multi-row kernel merges per chunk, within f32 reassociation
    (atol 2e-3); from 5 rows the matrix-core kernel takes P in bf16, within bf16 rounding (atol 1e-2)."""
    B, H, hd = 3, 20, 64
    d = H * hd
    dtype = torch.bfloat16
    k = torch.randn(B, H, S, hd, device="cuda").to(dtype)
    v = torch.randn(B, H, S, hd, device="cuda").to(dtype)
    q = (torch.randn(B * q_len, d, device="cuda") * 0.3).to(dtype)
    out = torch.empty(B * q_len, d, device="cuda", dtype=dtype)
    ws = torch.zeros(ops.cross_attn_workspace_bytes(B, q_len, H, hd, S) // 4 + 1, device="cuda")
    for _ in range(2):
        ops.cross_attn_step(q, B, q_len, H, hd, k, v, S, out, ws)
    one = torch.empty(B, d, device="cuda", dtype=dtype)
    ws1 = torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, hd, S) // 4 + 1, device="cuda")
    qv = q.view(B, q_len, d)
    for i in range(q_len):
        ops.cross_attn_step(qv[:, i].contiguous(), B, 1, H, hd, k, v, S, one, ws1)
        if q_len <= 4 and S <= 256:
            assert torch.equal(out.view(B, q_len, d)[:, i], one), i
        elif q_len <= 4:
            torch.testing.assert_close(out.view(B, q_len, d)[:, i].float(), one.float(), atol=2e-3, rtol=1e-2)
        else:
            torch.testing.assert_close(out.view(B, q_len, d)[:, i].float(), one.float(), atol=1e-2, rtol=1e-2)
    _check_cross_ws_rearmed(ws1, B * H, S)
    _check_cross_ws_rearmed(ws, B * q_len * H, S)


# ---------------------------------------------------------------- greedy step (processors + argmax)
def _random_history(rng, B, P, n, ts_begin, V, eos, pad):
    ids = np.zeros((B, P + n), np.int64)
    ids[:, :P] = [50258, 50266, 50360][:P] if P <= 3 else 0
    for b in range(B):
        for j in range(n):
            r = rng.random()
            ids[b, P + j] = rng.integers(ts_begin, V) if r < 0.4 else rng.integers(0, eos)
    ids[1, P + n - 2:] = [eos, pad] if n >= 2 else ids[1, P + n - 2:]
    return ids


@pytest.mark.parametrize("rt", [False, True])
@pytest.mark.parametrize("n_hist", [0, 1, 2, 5, 30])
def test_greedy_step_vs_oracle(rt, n_hist):
    from kwhisper.config import LARGE_V3, generation_constants
    from oracle.generate import process_logits

    gen = generation_constants(LARGE_V3)
    V = LARGE_V3.vocab_size
    B, P = 6, 3
    rng = np.random.default_rng(n_hist + 100 * rt)
    hist = _random_history(rng, B, P, n_hist, gen.timestamp_begin, V, gen.eos_token_id, gen.pad_token_id)
    logits = rng.standard_normal((B, V)).astype(np.float32) * 3
    logits[:, gen.timestamp_begin:] += 2.0 * (np.arange(B)[:, None] % 2)  # some rows favour timestamps
    gd = gen.to_dict()
    want = process_logits(hist, logits, gd, P, rt)
    L_now = hist.shape[1]
    ids = torch.zeros((B, 449), dtype=torch.int64, device="cuda")
    ids[:, :L_now] = torch.from_numpy(hist)
    cur = torch.tensor([L_now], dtype=torch.int32, device="cuda")
    unf = torch.ones(B, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    nun = torch.zeros(1, dtype=torch.int32, device="cuda")
    sup = torch.zeros(V, dtype=torch.uint8)
    sup[torch.tensor(gen.suppress_tokens)] = 1
    scores = torch.empty((B, V), device="cuda")
    lg = dev(logits)
    plan = ops.SamplerPlan(lg, sup.cuda(), torch.tensor(gen.begin_suppress_tokens, dtype=torch.int32, device="cuda"),
                           ids, cur, unf, cnt, nun, return_timestamps=rt, ts_begin=gen.timestamp_begin,
                           no_ts_id=gen.no_timestamps_token_id, eos_id=gen.eos_token_id, pad_id=gen.pad_token_id,
                           max_initial_ts=gen.max_initial_timestamp_index, max_length=448, begin_index=P,
                           scores_out=scores)
    plan()
    torch.cuda.synchronize()
    got = scores.cpu().numpy()
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(want))
    fin = [(hist[b, P:] == gen.eos_token_id).any() for b in range(B)]
    tok = ids[:, L_now].cpu().numpy()
    for b in range(B):
        exp_tok = gen.pad_token_id if fin[b] else int(np.argmax(want[b]))
        assert tok[b] == exp_tok
    assert int(cur.item()) == L_now + 1
    assert int(nun.item()) == int(unf.sum().item())


@pytest.mark.parametrize("rt", [False, True])
@pytest.mark.parametrize("n_hist", [0, 1, 7])
@pytest.mark.parametrize("B,V", [(32, 51866), (6, 51865), (3, 1000), (2, 9)])
def test_greedy_step_split_rows(rt, n_hist, B, V):
    """Split-row sampler (a row over 8 workgroups + last-arriver combine; with timestamps the probability-mass
    rule from merged per-slice log-sum-exps) == the one-workgroup kernel, token for token: ties (first
    index wins), EOS-finished rows, the begin-suppress step, timestamp pairing / monotonicity / initial
    rules, the text ban, and the cur_len / n_unfinished bookkeeping over repeated steps."""
    from kwhisper.config import LARGE_V3, generation_constants

    gen = generation_constants(LARGE_V3)
    P = 3
    rng = np.random.default_rng(1000 * n_hist + V + B + 7 * rt)
    eos = min(gen.eos_token_id, V - 4)
    ts_begin = gen.timestamp_begin if V > gen.timestamp_begin else V - 3
    no_ts = ts_begin - 1
    hist = rng.integers(0, eos, (B, P + n_hist))
    if n_hist:
        hist[0, P] = eos  # a finished row
        hist[1 % B, P:] = rng.integers(ts_begin, V, n_hist)  # a row of timestamps
    sup = torch.zeros(V, dtype=torch.uint8)
    sup[torch.tensor([t for t in gen.suppress_tokens if t < no_ts][:50] + [1])] = 1
    bsup = torch.tensor([0, min(220, V - 1)], dtype=torch.int32, device="cuda")
    outs = []
    for split in (False, True):
        ids = torch.zeros((B, 64), dtype=torch.int64, device="cuda")
        ids[:, : hist.shape[1]] = torch.from_numpy(hist)
        cur = torch.tensor([hist.shape[1]], dtype=torch.int32, device="cuda")
        unf = torch.ones(B, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        nun = torch.zeros(1, dtype=torch.int32, device="cuda")
        lg = torch.empty((B, V), device="cuda")
        ws = torch.zeros(ops.greedy_step_workspace_bytes(B) // 4 + 1, device="cuda") if split else None
        plan = ops.SamplerPlan(lg, sup.cuda(), bsup, ids, cur, unf, cnt, nun, return_timestamps=rt,
                               ts_begin=ts_begin, no_ts_id=no_ts, eos_id=eos, pad_id=gen.pad_token_id % V,
                               max_initial_ts=50 if rt else None, max_length=hist.shape[1] + 5, begin_index=P,
                               workspace=ws)
        srng = np.random.default_rng(7)
        for step in range(4):
            if rt:  # continuous scores (no exact ties between the log-sum-exp sides), some rows favour stamps
                x = (srng.standard_normal((B, V)) * 3).astype(np.float32)
                x[::2, ts_begin:] += 4.0 + step
            else:
                x = srng.integers(-3, 4, (B, V)).astype(np.float32)  # many ties
            lg.copy_(torch.from_numpy(x))
            plan()
        torch.cuda.synchronize()
        outs.append((ids.cpu().numpy(), int(cur.item()), unf.cpu().numpy(), int(nun.item()), int(cnt.item())))
        if split:
            assert not ws.view(torch.int32)[B * 64: B * 65].any()  # per-row counters back at zero
    (a_ids, a_cur, a_unf, a_nun, a_cnt), (b_ids, b_cur, b_unf, b_nun, b_cnt) = outs
    np.testing.assert_array_equal(a_ids, b_ids)
    assert (a_cur, a_nun, a_cnt) == (b_cur, b_nun, b_cnt) and (a_unf == b_unf).all()


@pytest.mark.parametrize("M", [32, 5, 1, 70, 320, 333])
@pytest.mark.parametrize("N,K", [(3840, 1280), (5120, 1280), (1280, 1280), (51866, 1280), (1152, 384), (51865, 384)])
def test_dec_linear_layernorm(M, N, K):
    """LayerNorm-fused STORE: gamma/beta folded into W and bias as the engine loads them, the rows'
    statistics computed in-kernel from the bf16 operand; against an fp32 reference of LN(x) W^T + b."""
    h = torch.randn(M, K, device="cuda") * 2 + 0.5
    hb = h.bfloat16()
    g = 1 + 0.1 * torch.randn(K, device="cuda")
    bb = 0.1 * torch.randn(K, device="cuda")
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    bias = torch.randn(N, device="cuda")
    Wf = (W.float() * g[None, :]).bfloat16()
    C = torch.empty(M, N, device="cuda")
    ops.DecLinearPlan(hb, ops.pack_weight(Wf), M, N, K, ln=(1e-5, ops.ln_colsum(Wf)), bias=bias + W.float() @ bb,
                      C=C)()
    xn = torch.nn.functional.layer_norm(hb.float(), (K,), g, bb, 1e-5).bfloat16()
    torch.testing.assert_close(C, _ref_gemm(xn, W, bias), atol=4e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 5, 32])
def test_dec_linear_ln_gelu_bf16(M):
    """The production fc1 variant: N 5120, K 1280, LayerNorm fused, exact-erf GELU, bf16 STORE,
    at decode row counts (<KTM=5, NCB=2, LNA> geometry), against fp32 GELU(LN(x) W^T + b)."""
    torch.manual_seed(M)
    N, K = 5120, 1280
    h = torch.randn(M, K, device="cuda") * 2 + 0.5
    hb = h.bfloat16()
    g = 1 + 0.1 * torch.randn(K, device="cuda")
    bb = 0.1 * torch.randn(K, device="cuda")
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    bias = 0.1 * torch.randn(N, device="cuda")
    Wf = (W.float() * g[None, :]).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.DecLinearPlan(hb, ops.pack_weight(Wf), M, N, K, ln=(1e-5, ops.ln_colsum(Wf)), bias=bias + W.float() @ bb,
                      C=C, gelu=True)()
    xn = torch.nn.functional.layer_norm(hb.float(), (K,), g, bb, 1e-5).bfloat16()
    ref = torch.nn.functional.gelu(_ref_gemm(xn, W, bias))
    err = (C.float() - ref).abs()
    print(f"fc1 LN+GELU bf16 M={M}: max err {err.max().item():.4f}")
    torch.testing.assert_close(C.float(), ref, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [64, 70, 320])
@pytest.mark.parametrize("N,K,mode", [(3840, 1280, "ln"), (1280, 1280, "resid"), (5120, 1280, "gelu_bf16"),
                                      (1152, 384, "ln"), (384, 1536, "resid")])
def test_dec_linear_rows_bitwise(M, N, K, mode):
    """More than 32 rows (prefill, beam rows) run weight-stationary workgroups over 32-row chunks: bit for
    bit the results of the same linear launched on each 32-row slice alone."""
    torch.manual_seed(M + N + K)
    x = (torch.randn(M, K, device="cuda") * 2 + 0.3).bfloat16()
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    Wp = ops.pack_weight(W)
    b = torch.randn(N, device="cuda")
    ws = torch.zeros(ops.dec_linear_workspace_bytes(N, K) // 4 + 1, device="cuda")
    h0 = torch.randn(M, N, device="cuda")

    def run(rows, r0):
        xs = x[r0:r0 + rows].contiguous()
        if mode == "resid":
            h = h0[r0:r0 + rows].clone()
            hb = torch.empty(rows, N, device="cuda", dtype=torch.bfloat16)
            ops.DecLinearPlan(xs, Wp, rows, N, K, bias=b, resid=(h, hb, N, 0), workspace=ws)()
            return h, hb
        if mode == "ln":
            C = torch.empty(rows, N, device="cuda")
            ops.DecLinearPlan(xs, Wp, rows, N, K, ln=(1e-5, ops.ln_colsum(W)), bias=b, C=C)()
            return (C,)
        C = torch.empty(rows, N, device="cuda", dtype=torch.bfloat16)
        ops.DecLinearPlan(xs, Wp, rows, N, K, bias=b, C=C, gelu=True, scale=0.5, scale_cols=N // 3)()
        return (C,)

    full = run(M, 0)
    for r0 in range(0, M, 32):
        part = run(min(32, M - r0), r0)
        for f, q in zip(full, part):
            assert torch.equal(f[r0:r0 + q.shape[0]], q), r0


@pytest.mark.parametrize("M", [32, 5, 70, 300])
@pytest.mark.parametrize("N,K", [(1280, 1280), (1280, 5120), (384, 1536)])
def test_dec_linear_resid(M, N, K):
    """RESID epilogue (h += x W^T + b, bf16 mirror); K 5120 exercises the K-split seam.  Run twice:
    bitwise identical (the seam counters come back to zero, the reduction order is fixed)."""
    W = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    A = torch.randn(M, K, device="cuda").bfloat16()
    h0 = torch.randn(M, N, device="cuda")
    Wp = ops.pack_weight(W)
    ws = torch.zeros(ops.dec_linear_workspace_bytes(N, K) // 4 + 1, device="cuda")
    outs = []
    for _ in range(2):
        h, hb = h0.clone(), torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ops.DecLinearPlan(A, Wp, M, N, K, bias=b, resid=(h, hb, N, 0), workspace=ws)()
        outs.append(h)
        assert torch.equal(hb, h.bfloat16())
    torch.testing.assert_close(outs[0], h0 + _ref_gemm(A, W, b), atol=2e-3, rtol=2e-3)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("B,q,d", [(3, 2, 384), (32, 1, 1280), (2, 4, 1280), (3, 1, 12)])
def test_embed_mirror(B, q, d):
    """h = tok_emb[id] + pos_emb[pos] in f32 and its bf16 mirror, bit for bit (the 16-B vector kernel for
    d % 8 == 0 -- r06 -- and the element kernel for d = 12)."""
    V = 1000
    tok = torch.randn(V, d, device="cuda").bfloat16()
    pos = torch.randn(448, d, device="cuda").bfloat16()
    ids = torch.randint(0, V, (B, 449), device="cuda")
    cur = torch.tensor([7], dtype=torch.int32, device="cuda")
    h = torch.empty(B * q, d, device="cuda")
    hb = torch.empty(B * q, d, device="cuda", dtype=torch.bfloat16)
    ops.embed(ids, B, q, cur, tok, pos, h, hb)
    ref = (tok[ids[:, 7 - q:7]].float() + pos[7 - q:7].float()).reshape(B * q, d)
    assert torch.equal(h, ref)
    assert torch.equal(hb, ref.bfloat16())


@pytest.mark.parametrize("B,V,K", [(32, 51866, 1280), (5, 51866, 1280), (1, 51865, 1280), (17, 51865, 384)])
def test_lm_greedy_equals_lm_head_then_sampler(B, V, K):
    """kw_dec_lm_greedy (the LM head and the greedy step in one launch, r06) == kw_dec_linear(LM head) followed by
    kw_greedy_step, over five steps: the same tokens (ties between duplicated weight rows -> the first index; the
    SuppressTokens mask; SuppressTokensAtBegin on the first step; a row finished by EOS emitting pad; max_length), the
    same cur_len / unfinished / n_unfinished bookkeeping, the logits bit for bit when stored, and the arrival counter
    back at zero after every launch."""
    torch.manual_seed(B + V + K)
    P = 3
    eos, pad = 50257, 50256
    W = (torch.randn(V, K, device="cuda") / K ** 0.5).bfloat16()
    W[51000] = W[eos]  # tie pairs: a later duplicate never wins over the earlier row
    W[2000:2010] = W[1000:1010]
    Wp = ops.pack_weight(W)
    cs = ops.ln_colsum(W)
    bias = 0.1 * torch.randn(V, device="cuda")
    bias[51000] = bias[eos]
    bias[2000:2010] = bias[1000:1010]
    sup = torch.zeros(V, dtype=torch.uint8, device="cuda")
    sup[torch.randint(0, V, (400,), device="cuda")] = 1
    sup[[eos, 51000, 1005, 2005]] = 0
    bsup = torch.tensor([220, eos], dtype=torch.int32, device="cuda")
    x_steps = [(torch.randn(B, K, device="cuda") * 2 + 0.3).bfloat16() for _ in range(5)]
    for b in range(0, B, 3):  # some rows strongly prefer EOS (tied with row 51000: EOS wins, the row finishes)
        x_steps[1][b] = (W[eos].float() * 8).bfloat16()
    for b in range(1, B, 3):  # ... and some the tied pair 1005 / 2005 (1005 wins)
        x_steps[2][b] = (W[1005].float() * 8).bfloat16()
    outs = []
    for fused in (False, True):
        ids = torch.zeros((B, 64), dtype=torch.int64, device="cuda")
        ids[:, :P] = torch.tensor([50258, 50266, 50360])
        cur = torch.tensor([P], dtype=torch.int32, device="cuda")
        unf = torch.ones(B, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        nun = torch.zeros(1, dtype=torch.int32, device="cuda")
        x = torch.empty(B, K, device="cuda", dtype=torch.bfloat16)
        logits = torch.full((B, V), float("nan"), device="cuda")
        logs = []
        if fused:
            ws = torch.zeros(ops.lm_greedy_workspace_bytes(B, V) // 4 + 1, device="cuda")
            plan = ops.LmGreedyPlan(x, Wp, B, V, K, ln=(1e-5, cs), bias=bias, suppress_mask=sup, begin_suppress=bsup,
                                    ids=ids, cur_len=cur, unfinished=unf, n_unfinished=nun, eos_id=eos, pad_id=pad,
                                    max_length=P + 4, begin_index=P, workspace=ws, logits=logits)
            steps = [plan]
        else:
            sws = torch.zeros(ops.greedy_step_workspace_bytes(B) // 4 + 1, device="cuda")
            steps = [ops.DecLinearPlan(x, Wp, B, V, K, ln=(1e-5, cs), bias=bias, C=logits),
                     ops.SamplerPlan(logits, sup, bsup, ids, cur, unf, cnt, nun, return_timestamps=False, ts_begin=50365,
                                     no_ts_id=50364, eos_id=eos, pad_id=pad, max_initial_ts=None, max_length=P + 4,
                                     begin_index=P, workspace=sws)]
        for xs in x_steps:
            x.copy_(xs)
            for f in steps:
                f()
            logs.append(logits.clone())
            if fused:
                torch.cuda.synchronize()
                assert int(ws.view(torch.int32)[0].item()) == 0  # arrival counter re-armed
        torch.cuda.synchronize()
        outs.append((ids.cpu(), int(cur.item()), unf.cpu(), int(nun.item()), logs))
    (a_ids, a_cur, a_unf, a_nun, a_logs), (b_ids, b_cur, b_unf, b_nun, b_logs) = outs
    assert torch.equal(a_ids, b_ids), (a_ids[:, P:P + 5], b_ids[:, P:P + 5])
    assert (a_cur, a_nun) == (b_cur, b_nun) and torch.equal(a_unf, b_unf)
    assert (a_ids[:, P:P + 5] == eos).any() and (a_ids[:, P:P + 5] == pad).any()  # EOS finished some rows
    if B > 1:
        assert (a_ids[:, P + 2] == 1005).any() and not (a_ids[:, P:P + 5] == 2005).any()
    for la, lb in zip(a_logs, b_logs):
        assert torch.equal(la, lb)


@pytest.mark.parametrize("rt", [False, True])
@pytest.mark.parametrize("R,V,k,n_hist,adv", [(10, 51865, 10, 0, False), (10, 51865, 10, 5, False),
                                              (40, 51866, 6, 3, False), (4, 900, 16, 2, False),
                                              (12, 51866, 10, 2, True)])
def test_beam_logprobs_split_rows(rt, R, V, k, n_hist, adv):
    """kw_beam_logprobs split over 8 workgroups per row == the one-workgroup kernel: the same k candidate
    tokens per row in the same order, log-probs equal up to the normaliser's summation order.  ``adv``:
    logits on a 0.5 grid (ties broken by token), +-0.0 values, and rows whose best tokens all sit in one
    thread's registers of one slice (a lane that wins more rounds than its 3-key cache holds)."""
    import ctypes

    from kwhisper import _lib as L
    from kwhisper.config import LARGE_V3, generation_constants

    gen = generation_constants(LARGE_V3)
    P = 3
    rng = np.random.default_rng(R * 7 + V + k + n_hist + 100 * rt)
    eos = min(gen.eos_token_id, V - 4)
    ts_begin = gen.timestamp_begin if V > gen.timestamp_begin else V - 3
    hist = rng.integers(0, eos, (R, P + n_hist))
    if n_hist:
        hist[1, P:] = rng.integers(ts_begin, V, n_hist)
    ids = torch.zeros((R, 64), dtype=torch.int64, device="cuda")
    ids[:, : hist.shape[1]] = torch.from_numpy(hist)
    cur = torch.tensor([hist.shape[1]], dtype=torch.int32, device="cuda")
    sup = torch.zeros(V, dtype=torch.uint8, device="cuda")
    sup[1] = 1
    bsup = torch.tensor([0, 7], dtype=torch.int32, device="cuda")
    done = torch.zeros(1, dtype=torch.int32, device="cuda")
    x = (rng.standard_normal((R, V)) * 3).astype(np.float32)
    x[::2, ts_begin:] += 3.0
    if adv:
        x = np.round(x * 2) / 2
        x[:, 5:40:3] = -0.0
        per = (V + 7) // 8
        for r in range(R):  # slice r % 8, thread 17: tokens v0 + 17 + 512 u
            v0 = (r % 8) * per
            toks = [v0 + 17 + 512 * u for u in range(16) if v0 + 17 + 512 * u < min(V, v0 + per)]
            x[r, toks] = 30.0 - (np.arange(len(toks)) % 3)
    lg = torch.from_numpy(x).cuda()
    res = []
    for split in (False, True):
        cv = torch.empty((R, k), device="cuda")
        ci = torch.empty((R, k), dtype=torch.int32, device="cuda")
        ws = torch.zeros(ops.beam_logprobs_workspace_bytes(R) // 4 + 1, device="cuda") if split else None
        a = L.BeamLogprobsArgs()
        a.logits, a.R, a.V = lg.data_ptr(), R, V
        a.suppress_mask, a.begin_suppress, a.n_begin_suppress = sup.data_ptr(), bsup.data_ptr(), 2
        a.return_timestamps, a.ts_begin, a.no_ts_id, a.eos_id = int(rt), ts_begin, ts_begin - 1, eos
        a.max_initial_ts = 50
        a.ids, a.ids_stride, a.cur_len, a.begin_index, a.k = ids.data_ptr(), 64, cur.data_ptr(), P, k
        a.cand_val, a.cand_idx, a.done = cv.data_ptr(), ci.data_ptr(), done.data_ptr()
        a.workspace = ws.data_ptr() if ws is not None else None
        a.ws_bytes = ws.numel() * 4 if ws is not None else 0
        for _ in range(2):
            L.check(L.load().kw_beam_logprobs(ctypes.byref(a), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                    "kw_beam_logprobs")
        torch.cuda.synchronize()
        res.append((cv.cpu().numpy(), ci.cpu().numpy()))
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_allclose(res[0][0], res[1][0], rtol=1e-6, atol=1e-5)


# ---------------------------------------------------------------- fused QKV projection + self-attention step
@pytest.mark.parametrize("M,d,H", [(32, 1280, 20), (7, 1280, 20), (1, 384, 6), (32, 384, 6)])
@pytest.mark.parametrize("L", [1, 5, 33, 128, 200, 256])
def test_qkv_self_fused_matches_two_launches(M, d, H, L):
    """kw_dec_qkv_self vs kw_dec_linear(qkv, LayerNorm fused, q scaled) then kw_self_attn_step(q_len 1): both
    caches bit for bit (the projection is the same arithmetic; the new row appended at L - 1), the attention
    output within bf16 rounding of an fp32 softmax over the same q / K / V (its keys are grouped in 16-slot
    passes, the unfused kernel's in 32 slots) and no further from it than the unfused output; positions L = 1
    (nothing cached) .. 256 (the largest it takes); deterministic; the workspace comes back re-armed (every
    granule tag 0, the error word 0), so a second launch on it gives the same result."""
    torch.manual_seed(M * 1000 + L + d)
    t_max, eps = 448, 1e-5
    hb = torch.randn(M, d, device="cuda").bfloat16()
    W = (torch.randn(3 * d, d, device="cuda") / d ** 0.5).bfloat16()
    packed, colsum = ops.pack_weight(W), ops.ln_colsum(W)
    bias = torch.randn(3 * d, device="cuda") * 0.1
    kc = torch.randn(M, H, t_max, 64, device="cuda").bfloat16()
    vc = torch.randn(M, H, t_max, 64, device="cuda").bfloat16()
    cur = torch.tensor([L], dtype=torch.int32, device="cuda")
    qkv = torch.empty(M, 3 * d, device="cuda", dtype=torch.bfloat16)
    lws = torch.zeros(ops.dec_linear_workspace_bytes(3 * d, d) // 4 + 1, device="cuda")
    ops.DecLinearPlan(hb, packed, M, 3 * d, d, ln=(eps, colsum), bias=bias, C=qkv, scale=0.125, scale_cols=d,
                      workspace=lws)()
    kc1, vc1 = kc.clone(), vc.clone()
    out1 = torch.empty(M, d, device="cuda", dtype=torch.bfloat16)
    sws = torch.zeros(ops.self_attn_workspace_bytes(M, H, t_max) // 4 + 1, device="cuda")
    ops.self_attn_step(qkv, M, 1, H, 64, kc1, vc1, t_max, cur, out1, sws)
    q = qkv[:, :d].float().view(M, H, 1, 64)
    sc = q @ kc1[:, :, :L].float().transpose(-1, -2)
    ref = (torch.softmax(sc, -1) @ vc1[:, :, :L].float()).view(M, d)
    err1 = (out1.float() - ref).abs().max().item()
    assert ops.qkv_self_supported(M, d, H)
    qws = torch.zeros(ops.qkv_self_workspace_bytes(M, d) // 4 + 1, device="cuda")
    first = None
    for rep in range(2):
        kc2, vc2 = kc.clone(), vc.clone()
        out2 = torch.full((M, d), 7.0, device="cuda", dtype=torch.bfloat16)
        ops.QkvSelfPlan(hb, packed, M, d, H, ln=(eps, colsum), bias=bias, scale=0.125, k_cache=kc2, v_cache=vc2,
                        t_max=t_max, cur_len=cur, out=out2, workspace=qws)()
        torch.cuda.synchronize()
        assert int(qws.view(torch.int32).abs().sum()) == 0, "granules not re-armed / a poll timed out"
        assert torch.equal(kc2, kc1) and torch.equal(vc2, vc1), rep
        diff = (out2.float() - ref).abs()
        assert bool((diff <= 8e-3 * (1 + ref.abs())).all()), (rep, diff.max().item())
        assert diff.max().item() <= 2 * err1 + 1e-3, (diff.max().item(), err1)
        if first is None:
            first = out2.clone()
        else:
            assert torch.equal(out2, first)


# ---------------------------------------------------------------- fused cross-attention query + step
@pytest.mark.parametrize("M,d,H,S", [(32, 1280, 20, 1500), (7, 1280, 20, 1500), (1, 384, 6, 1500),
                                     (32, 384, 6, 500), (5, 512, 8, 240), (32, 512, 8, 1500)])
def test_xq_cross_fused_matches_two_launches(M, d, H, S):
    """kw_dec_xq_cross == kw_dec_linear(xq, LayerNorm fused, every column scaled) then kw_cross_attn_step(q_len 1),
    bit for bit (the projection is dec_linear's arithmetic on virtual waves, the attention cross_attn_dma_kernel's),
    and close to an fp32 softmax over the same query and K / V; chunk counts 6, 2 and 1 (S = 1500, 500, 240);
    repeated launches on one workspace, which comes back zero (every query and chunk-partial granule re-armed,
    the error word 0)."""
    torch.manual_seed(M * 7 + d + S)
    eps = 1e-5
    hb = torch.randn(M, d, device="cuda").bfloat16()
    W = (torch.randn(d, d, device="cuda") / d ** 0.5).bfloat16()
    packed, colsum = ops.pack_weight(W), ops.ln_colsum(W)
    bias = torch.randn(d, device="cuda") * 0.1
    k = torch.randn(M, H, S, 64, device="cuda").bfloat16()
    v = torch.randn(M, H, S, 64, device="cuda").bfloat16()
    qx = torch.empty(M, d, device="cuda", dtype=torch.bfloat16)
    lws = torch.zeros(ops.dec_linear_workspace_bytes(d, d) // 4 + 1, device="cuda")
    ops.DecLinearPlan(hb, packed, M, d, d, ln=(eps, colsum), bias=bias, C=qx, scale=0.125, scale_cols=d,
                      workspace=lws)()
    out1 = torch.empty(M, d, device="cuda", dtype=torch.bfloat16)
    cws = torch.zeros(ops.cross_attn_workspace_bytes(M, 1, H, 64, S) // 4 + 1, device="cuda")
    ops.cross_attn_step(qx, M, 1, H, 64, k, v, S, out1, cws)
    qq = qx.float().view(M, 1, H, 64).permute(0, 2, 1, 3)
    ref = (torch.softmax(qq @ k.float().transpose(-1, -2), -1) @ v.float()).permute(0, 2, 1, 3).reshape(M, d)
    err1 = (out1.float() - ref).abs().max().item()
    assert ops.xq_cross_supported(M, d, H, S)
    ws = torch.zeros(ops.xq_cross_workspace_bytes(M, d, H, S) // 4 + 1, device="cuda")
    for rep in range(3):
        out2 = torch.full((M, d), 7.0, device="cuda", dtype=torch.bfloat16)
        ops.XqCrossPlan(hb, packed, M, d, H, ln=(eps, colsum), bias=bias, scale=0.125, k=k, v=v, S=S, out=out2,
                        workspace=ws)()
        torch.cuda.synchronize()
        assert int(ws.view(torch.int32).abs().sum()) == 0, "granules not re-armed / a poll timed out"
        assert torch.equal(out2, out1), (rep, (out2.float() - out1.float()).abs().max().item())
    assert err1 < 2e-2, err1


def test_xq_cross_rejects_what_it_does_not_cover():
    assert not ops.xq_cross_supported(33, 1280, 20, 1500)  # more rows than one 32-row tile
    assert not ops.xq_cross_supported(4, 1280, 16, 1500)   # head_dim != 64
    assert not ops.xq_cross_supported(4, 1280, 20, 200)    # chunks under 225 keys (the two-launch path's)
    assert not ops.xq_cross_supported(4, 1536, 24, 1500)   # K beyond dec_linear's 8 waves x 5 k-tiles


def test_qkv_self_rejects_what_it_does_not_cover():
    assert not ops.qkv_self_supported(33, 1280, 20)  # more rows than one 32-row tile
    assert not ops.qkv_self_supported(4, 1280, 16)   # head_dim != 64
