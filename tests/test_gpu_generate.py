"""End-to-end parity of the MI355X generate() against golden vectors from the reference path.

fp32 engine: greedy token matrices must be bit-exact with transformers 5.15.0 (CPU, fp32) for every
prompt / timestamp / padding mode of tests/golden/tiny_fp32.npz and for large-v3 / kotoba-v2.0.
bf16 engine (the performance path): per-step teacher-forced logits within a stated tolerance of the
fp32 reference, and greedy tokens equal wherever the reference's top-1/top-2 margin exceeds the
bf16 noise floor.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from kwhisper.config import KOTOBA_V2, LARGE_V3, TINY, generation_constants  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict  # noqa: E402

from _util import BEAM_MODES, TINY_MODES, oracle_features  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(shape, dtype, pad=None):
    from kwhisper.generation import KWhisperForConditionalGeneration

    return KWhisperForConditionalGeneration.from_state_dict(
        shape, synthetic_state_dict(shape, 0), dtype=dtype, generation_config=generation_constants(shape, pad))


@pytest.fixture(scope="module")
def tiny32():
    return _model(TINY, torch.float32)


@pytest.fixture(scope="module")
def tiny16():
    return _model(TINY, torch.bfloat16)


def test_tiny_fp32_encoder(gold, tiny32):
    g = gold("tiny_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    enc = tiny32.get_encoder()(feats).last_hidden_state.cpu().numpy()
    np.testing.assert_allclose(enc[:, ::50, :], g["enc_slice"], atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize("mode", sorted(TINY_MODES))
def test_tiny_fp32_generate_bitexact(gold, tiny32, mode):
    g = gold("tiny_fp32")
    kw, pad = TINY_MODES[mode]
    kw = dict(kw)
    model = tiny32
    if pad is not None:
        model.generation_config = generation_constants(TINY, pad)
    try:
        feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
        kw.setdefault("max_length", int(g["max_length"]))
        res = model.generate(feats, **kw)
        toks = res["sequences"] if isinstance(res, dict) else res
        np.testing.assert_array_equal(toks.cpu().numpy(), g[f"{mode}_tokens"])
    finally:
        model.generation_config = generation_constants(TINY)


@pytest.mark.parametrize("mode", sorted(BEAM_MODES))
def test_tiny_fp32_beam_bitexact(gold, tiny32, mode):
    """Device beam search (kw_beam_logprobs + kw_beam_select, slot-table self-attention) against HF beam
    search: EOS finishing, length penalty, early_stopping True / "never", timestamps; bit-exact tokens."""
    g = gold("tiny_beam_fp32")
    kw, eos = BEAM_MODES[mode]
    gen = generation_constants(TINY)
    if eos is not None:
        gen.eos_token_id = eos
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    toks = tiny32.generate(feats, generation_config=gen, **kw)
    np.testing.assert_array_equal(toks.cpu().numpy(), g[f"{mode}_tokens"])


def test_tiny_bf16_beam_runs(gold, tiny16):
    """bf16 engine: beam search with timestamps runs end to end (graph-replayed) with valid ids."""
    g = gold("tiny_beam_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    toks = tiny16.generate(feats, language="ja", task="transcribe", return_timestamps=True, num_beams=5,
                           max_length=40).cpu().numpy()
    assert toks.shape[0] == 4 and 0 < toks.shape[1] <= 40
    assert toks.min() >= 0 and toks.max() < TINY.vocab_size


def _tf_logprobs(eng, enc_row, seq, P):
    """Per-token log-softmax of the teacher-forced logits of ``seq`` (prompt + generated) at positions P.."""
    sess = eng.new_session(1, enc_row)
    t = torch.as_tensor(seq, dtype=torch.int64)[None]
    lg = sess.teacher_forced_logits(t, P)[0, : t.shape[1] - P].float()
    lp = torch.log_softmax(lg, -1)
    return lp.gather(-1, t[0, P:].cuda()[:, None])[:, 0].double().cpu().numpy()


@pytest.mark.parametrize("mode", ["beam3_eos", "beam2_eos_never"])
def test_tiny_bf16_beam_rescored(gold, tiny32, tiny16, mode):
    """bf16 beam search with beams that finish on EOS (length penalty 1.0 / 2.0, early_stopping False / "never"):
    every item's chosen hypothesis, rescored by the fp32 engine (bit-exact to HF beam search above) with HF's
    finished-beam score -- sum of log-probs / generated_len ** length_penalty (TF/generation/utils.py:3182) --
    is as good as HF fp32's choice within the bf16 scoring noise of the two hypotheses."""
    g = gold("tiny_beam_fp32")
    kw, eos = BEAM_MODES[mode]
    gen = generation_constants(TINY)
    gen.eos_token_id = eos
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    t16 = tiny16.generate(feats, generation_config=gen, **kw).cpu().numpy()
    t32 = g[f"{mode}_tokens"]
    prompt = [gen.decoder_start_token_id, gen.lang_to_id["<|ja|>"], gen.task_to_id["transcribe"],
              gen.no_timestamps_token_id]
    P, max_new, lp_pen = len(prompt), kw["max_length"], kw.get("length_penalty", 1.0)
    e32 = tiny32.engine.encode(feats).view(4, 1500, -1)
    e16 = tiny16.engine.encode(feats).view(4, 1500, -1)

    def hyp(row):
        r = [int(x) for x in row]
        while r and r[-1] == gen.pad_token_id:
            r.pop()
        return prompt + r + ([eos] if len(r) < max_new else [])

    same = 0
    for b in range(4):
        h16, h32 = hyp(t16[b]), hyp(t32[b])
        s = {}
        for name, h in (("h16", h16), ("h32", h32)):
            lp32 = _tf_logprobs(tiny32.engine, e32[b].reshape(1500, -1), h, P)
            lp16 = _tf_logprobs(tiny16.engine, e16[b].reshape(1500, -1), h, P)
            n = len(h) - P
            s[name] = (lp32.sum() / n ** lp_pen, lp16.sum() / n ** lp_pen)
        tol = abs(s["h16"][1] - s["h16"][0]) + abs(s["h32"][1] - s["h32"][0]) + 1e-4
        same += h16 == h32
        print(f"\ntiny bf16 {mode} item {b}: same hypothesis {h16 == h32}; fp32 score of the bf16 choice "
              f"{s['h16'][0]:.5f} vs HF fp32's {s['h32'][0]:.5f} (tolerance {tol:.5f})")
        assert s["h16"][0] >= s["h32"][0] - tol
    print(f"tiny bf16 {mode}: {same}/4 items chose HF fp32's hypothesis")


def test_tiny_fp32_logits(gold, tiny32):
    g = gold("tiny_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    eng = tiny32.engine
    sess = eng.new_session(feats.shape[0], eng.encode(feats))
    seq = torch.from_numpy(g["greedy_sequences"])
    lg = sess.teacher_forced_logits(seq[:, :-1], 4).cpu()
    idx, val = g["greedy_logits_top_idx"], g["greedy_logits_top_val"]
    got = torch.gather(lg[:, : idx.shape[1]], -1, torch.from_numpy(idx.astype(np.int64))).numpy()
    np.testing.assert_allclose(got, val, atol=1e-3, rtol=0)  # north-star: logits within 1e-3 fp32


def test_tiny_bf16_logits_and_tokens(gold, tiny16):
    """bf16 tiny: teacher-forced logits and margin-gated greedy tokens."""
    g = gold("tiny_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    eng = tiny16.engine
    sess = eng.new_session(feats.shape[0], eng.encode(feats))
    seq = torch.from_numpy(g["greedy_sequences"])
    lg = sess.teacher_forced_logits(seq[:, :-1], 4).cpu()
    idx, val = g["greedy_logits_top_idx"], g["greedy_logits_top_val"]
    got = torch.gather(lg[:, : idx.shape[1]], -1, torch.from_numpy(idx.astype(np.int64))).numpy()
    err = np.abs(got - val)
    print("tiny bf16 teacher-forced logit err: max %.4f mean %.4f" % (err.max(), err.mean()))
    assert err.max() < 0.25 and err.mean() < 0.03   # bf16 weights/activations, f32 accumulation
    toks = tiny16.generate(feats, language="ja", task="transcribe", max_length=128).cpu().numpy()
    want = g["greedy_tokens"]
    margin = g["greedy_margin"]
    for b in range(want.shape[0]):
        # tokens must agree up to the first step whose reference margin is within bf16 noise
        unsafe = np.nonzero(margin[b] < 0.1)[0]
        upto = unsafe[0] if unsafe.size else want.shape[1]
        np.testing.assert_array_equal(toks[b, :upto], want[b, :upto])


@pytest.mark.parametrize("shape,tag", [(LARGE_V3, "large_v3_fp32"), (KOTOBA_V2, "kotoba_v2_fp32")])
def test_large_fp32_bitexact(gold, shape, tag):
    g = gold(tag)
    model = _model(shape, torch.float32)
    feats = torch.from_numpy(oracle_features(shape, g["cases"])).cuda()
    enc = model.get_encoder()(feats).last_hidden_state.cpu().numpy()
    np.testing.assert_allclose(enc[:, ::50, :], g["enc_slice"], atol=5e-4, rtol=1e-3)
    toks = model.generate(feats, language="ja", task="transcribe", max_length=int(g["max_length"]))
    np.testing.assert_array_equal(toks.cpu().numpy(), g["greedy_tokens"])
    if "greedy_ts_tokens" in g:
        toks = model.generate(feats, language="ja", task="transcribe", return_timestamps=True, max_length=24)
        np.testing.assert_array_equal(toks.cpu().numpy(), g["greedy_ts_tokens"])
    del model
    torch.cuda.empty_cache()


def test_large_bf16_vs_reference(gold):
    """bf16 large-v3 against the fp32 HF fixture."""
    g = gold("large_v3_fp32")
    model = _model(LARGE_V3, torch.bfloat16)
    feats = torch.from_numpy(oracle_features(LARGE_V3, g["cases"])).cuda()
    eng = model.engine
    enc = eng.encode(feats)
    e = enc.view(2, 1500, 1280).float().cpu().numpy()[:, ::50, :]
    rel = np.abs(e - g["enc_slice"]).max() / np.abs(g["enc_slice"]).max()
    print("large-v3 bf16 encoder rel err", rel)
    assert rel < 0.05
    sess = eng.new_session(2, enc)
    seq = torch.from_numpy(g["greedy_sequences"])
    lg = sess.teacher_forced_logits(seq[:, :-1], 4).cpu()
    idx, val = g["greedy_logits_top_idx"], g["greedy_logits_top_val"]
    got = torch.gather(lg[:, : idx.shape[1]], -1, torch.from_numpy(idx.astype(np.int64))).numpy()
    err = np.abs(got - val)
    print("large-v3 bf16 teacher-forced logit err: max %.4f mean %.4f" % (err.max(), err.mean()))
    assert err.max() < 0.35 and err.mean() < 0.03  # the same bars as config 3 at B = 32 (test_gpu_workloads.py)
    del model, sess
    torch.cuda.empty_cache()


@pytest.mark.parametrize("ts", [False, True])
def test_generate_multitask_reuses_encoder(gold, tiny32, ts):
    """SURVEY §8f row 4 (run_pseudo_labelling_v3.py:309-321): generate_multitask == one generate() per
    (language, task), bit-exact, with the first-pass encoder run once for all prompts (later seek-loop
    passes re-encode shifted mel per prompt, as the reference does)."""
    g = gold("tiny_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    tasks = [("ja", "transcribe"), ("ja", "translate"), ("en", "transcribe")]
    eng = tiny32.engine
    calls = []
    orig = eng.encode

    def counting(mel):
        calls.append(mel.shape[0])
        return orig(mel)

    eng.encode = counting
    try:
        want = [tiny32.generate(feats, language=l, task=t, return_timestamps=ts).cpu() for l, t in tasks]
        n_separate = len(calls)
        calls.clear()
        got = tiny32.generate_multitask(feats, tasks, return_timestamps=ts)
        n_multi = len(calls)
        again = tiny32.generate(feats, language="ja", task="transcribe", return_timestamps=ts).cpu()
    finally:
        del eng.encode
    for a, b in zip(got, want):
        np.testing.assert_array_equal(a.cpu().numpy(), b.numpy())
    np.testing.assert_array_equal(again.numpy(), want[0].numpy())  # the memo does not leak into plain calls
    assert n_multi == n_separate - (len(tasks) - 1), (n_multi, n_separate)


def test_tiny_fp32_longform_bitexact(gold, tiny32):
    """Long-form generate (> 3000 mel frames: the seek loop re-encodes shifted 30 s windows,
    generation_whisper.py:785-903) == transformers on the same features: batched with an attention mask
    (tokens and segments), and one clip without a mask."""
    from _util import longform_inputs, segments_of

    g = gold("tiny_longform_fp32")
    feats, mask, one = longform_inputs(g["clips"])  # oracle log-mel (same tokens as HF's features)
    res = tiny32.generate(torch.from_numpy(feats).cuda(), attention_mask=torch.from_numpy(mask).cuda(),
                          language="ja", task="transcribe", return_timestamps=True, return_segments=True)
    np.testing.assert_array_equal(res["sequences"].cpu().numpy(), g["long_ts_segments_tokens"])
    want = segments_of(g["long_ts_segments_segments"])
    got = [[(s["start"], s["end"], len(s["tokens"])) for s in row] for row in res["segments"]]
    assert [[x[2] for x in r] for r in got] == [[x[2] for x in r] for r in want]
    for rg, rw in zip(got, want):
        np.testing.assert_allclose([x[:2] for x in rg], [x[:2] for x in rw], atol=1e-9)
    plain = tiny32.generate(torch.from_numpy(feats).cuda(), attention_mask=torch.from_numpy(mask).cuda(),
                            language="ja", task="transcribe", return_timestamps=True)
    np.testing.assert_array_equal(plain.cpu().numpy(), g["long_ts_tokens"])
    single = tiny32.generate(torch.from_numpy(one).cuda(), language="ja", task="transcribe", return_timestamps=True)
    np.testing.assert_array_equal(single.cpu().numpy(), g["long_single_tokens"])


def test_torch_ops_decode_graph_matches_ctypes(gold):
    """SURVEY §8b boundary: the bf16 engine launched through torch.ops.kw (the default path) -- greedy
    generate() with its prefill and step captured into hipGraphs, beam search, teacher-forced logits --
    is bit for bit the engine launched through the ctypes binding of the same C ABI."""
    from kwhisper import ops

    g = gold("tiny_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    seq = torch.from_numpy(g["greedy_sequences"])
    res = {}
    old = ops.backend()
    try:
        for be in ("torch", "ctypes"):
            ops.set_backend(be)
            m = _model(TINY, torch.bfloat16)  # fresh plans, sessions and graph captures per backend
            toks = m.generate(feats, language="ja", task="transcribe", max_length=64).cpu()
            beam = m.generate(feats, language="ja", task="transcribe", num_beams=3, max_length=24).cpu()
            sess = m.engine.new_session(feats.shape[0], m.engine.encode(feats))
            lg = sess.teacher_forced_logits(seq[:, :12], 4).cpu()
            res[be] = (toks, beam, lg)
            del m, sess
    finally:
        ops.set_backend(old)
    for a, b in zip(res["torch"], res["ctypes"]):
        assert torch.equal(a, b)


def test_torch_ops_trace_under_torch_compile():
    """The custom ops are visible to torch.compile (fake implementations registered): a compiled function
    calling torch.ops.kw.layernorm / attention traces with fullgraph=True and equals the eager call."""
    from kwhisper import _lib

    kw = _lib.load_torch_ops()
    B, H, T, hd = 2, 4, 96, 64
    qkv = (torch.randn(3 * B * H * T * hd, device="cuda")).bfloat16()
    x = torch.randn(B * T, H * hd, device="cuda")
    gam, bet = torch.randn(H * hd, device="cuda"), torch.randn(H * hd, device="cuda")

    def f(qkv, x):
        out = torch.empty(B * T, H * hd, device="cuda", dtype=torch.bfloat16)
        kw.attention(qkv, B, H, T, hd, out)
        y = torch.empty_like(x)
        kw.layernorm(x, gam, bet, 1e-5, y, None)
        return out.float().sum() + y.sum(), out, y

    eager = f(qkv, x.clone())
    comp = torch.compile(f, fullgraph=True, backend="aot_eager")(qkv, x.clone())
    for a, b in zip(eager, comp):
        assert torch.equal(a, b)


def test_fused_decode_blocks_generate(gold):
    """The bf16 engine's greedy decode with the fused blocks (kw_dec_qkv_self and kw_dec_xq_cross, the default)
    vs the two-launch plans (fuse_qkv_self=False, fuse_xq_cross=False): the fused self-attention sums its keys in
    another grouping (bf16 rounding apart; the cross block is bitwise), so the tokens are compared margin-gated on the two-launch plan's own teacher-forced logits (equal up
    to each row's first step whose top-1/top-2 margin is below 0.05) and the teacher-forced logits on the golden
    sequences agree within 0.1 (max) / 0.01 (mean) -- a quarter of the bf16-vs-fp32 bars of
    test_tiny_bf16_logits_and_tokens; the fused plan really ran (fused_last).  (The encoder output is a per-engine buffer:
    every session is built on a fresh encode.)"""
    from kwhisper.engine import WhisperEngine
    from kwhisper.generation import KWhisperForConditionalGeneration

    g = gold("tiny_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"])).cuda()
    sd = synthetic_state_dict(TINY, 0)

    def mk(fuse):
        return KWhisperForConditionalGeneration(WhisperEngine(TINY, sd, dtype=torch.bfloat16,
                                                              generation_config=generation_constants(TINY),
                                                              fuse_qkv_self=fuse, fuse_xq_cross=fuse))

    fused, plain = mk(True), mk(False)
    compared = 0
    for ts in (False, True):
        a = fused.generate(feats, language="ja", task="transcribe", max_length=64, return_timestamps=ts).cpu()
        b = plain.generate(feats, language="ja", task="transcribe", max_length=64, return_timestamps=ts).cpu()
        P = 3 if ts else 4
        lb = plain.engine.new_session(4, plain.engine.encode(feats)).teacher_forced_logits(b, P).float().cpu()
        top2 = lb.topk(2, -1).values
        margin = (top2[..., 0] - top2[..., 1]).numpy()
        T = min(a.shape[1], b.shape[1])
        for r in range(b.shape[0]):
            unsafe = np.nonzero(margin[r, :T - P] < 0.05)[0]
            upto = P + (int(unsafe[0]) if unsafe.size else T - P)
            assert torch.equal(a[r, :upto], b[r, :upto]), (ts, r, upto)
            compared += upto - P
    assert compared > 0
    assert fused._sessions[(4, 1)].fused_last and not plain._sessions[(4, 1)].fused_last
    tags = {getattr(p, "tag", None) for p in fused._sessions[(4, 1)]._step_plans(1, fused=True)}
    assert {"qkv_self", "xq_cross"} <= tags, tags
    assert not {"qkv_self", "xq_cross"} & {getattr(p, "tag", None) for p in plain._sessions[(4, 1)]._step_plans(1)}
    seq = torch.from_numpy(g["greedy_sequences"])
    la = fused.engine.new_session(4, fused.engine.encode(feats)).teacher_forced_logits(seq[:, :-1], 4).float()
    lb = plain.engine.new_session(4, plain.engine.encode(feats)).teacher_forced_logits(seq[:, :-1], 4).float()
    diff = (la - lb).abs()
    print(f"fused vs two-launch: {compared} tokens compared; teacher-forced logits max diff {diff.max().item():.4g} "
          f"mean {diff.mean().item():.3g} (range {lb.abs().max().item():.3g})")
    assert diff.max().item() < 0.1 and diff.mean().item() < 0.01  # measured: max 0.025, mean 0.0015


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_encoder_streams_bitwise(tiny16, tiny32, dtype):
    """The encoder as row blocks on side streams (engine.encoder_streams, default 2; engine._encode_split) writes
    bitwise the one-pass encoder's rows -- also for a batch that does not split evenly (B = 5: 3 + 2 rows)."""
    eng = (tiny16 if dtype == torch.bfloat16 else tiny32).engine
    g = torch.Generator(device="cuda").manual_seed(11)
    mel = torch.randn(5, TINY.num_mel_bins, TINY.n_frames, device="cuda", generator=g) * 0.5
    old = eng.encoder_streams
    try:
        eng.encoder_streams = 1
        ref = eng.encode(mel).clone()
        for parts in (2, 3):
            eng.encoder_streams = parts
            got = eng.encode(mel)
            torch.cuda.synchronize()
            assert torch.equal(got.view(torch.int16) if dtype == torch.bfloat16 else got,
                               ref.view(torch.int16) if dtype == torch.bfloat16 else ref), parts
    finally:
        eng.encoder_streams = old


@pytest.mark.parametrize("ts", [False, True])
def test_prefill_streams_tokens_identical(tiny16, ts):
    """The greedy prefill as two row views on side streams (WhisperEngine.prefill_streams, default 2) gives
    generate() exactly the one-pass prefill's tokens (B = 6: two views of 3 rows), with and without timestamps."""
    g = torch.Generator(device="cuda").manual_seed(5)
    feats = torch.randn(6, TINY.num_mel_bins, TINY.n_frames, device="cuda", generator=g) * 0.5
    kw = dict(language="ja", task="transcribe", return_timestamps=ts, max_length=24)
    out = {}
    eng = tiny16.engine
    try:
        for parts in (2, 1):
            eng.prefill_streams = parts
            out[parts] = tiny16.generate(feats, **kw).cpu()
    finally:
        eng.prefill_streams = 2
    assert torch.equal(out[1], out[2])


@pytest.mark.parametrize("ts,eos", [(False, None), (True, None), (False, 7656)])
def test_steps_per_replay_tokens_identical(tiny16, ts, eos):
    """Two greedy steps per hipGraph replay (WhisperEngine.steps_per_replay, default 2) give exactly the tokens of
    one step per replay -- also when rows finish early on EOS (the host stop check's lag is kept in steps) and for
    an odd number of remaining steps (max_length 25: the last step replays the one-step graph)."""
    g = torch.Generator(device="cuda").manual_seed(9)
    feats = torch.randn(6, TINY.num_mel_bins, TINY.n_frames, device="cuda", generator=g) * 0.5
    gen = generation_constants(TINY)
    if eos is not None:
        gen.eos_token_id = eos
    kw = dict(language="ja", task="transcribe", return_timestamps=ts, max_length=25, generation_config=gen)
    out = {}
    eng = tiny16.engine
    try:
        for k in (2, 1, 3):
            eng.steps_per_replay = k
            out[k] = tiny16.generate(feats, **kw).cpu()
    finally:
        eng.steps_per_replay = 2
    assert torch.equal(out[1], out[2]) and torch.equal(out[1], out[3])


@pytest.mark.parametrize("eos", [None, 7656])
def test_lm_greedy_tokens_identical(tiny16, eos):
    """The LM head and the greedy step fused into one launch (kw_dec_lm_greedy, WhisperEngine.fuse_lm_greedy, the
    default without timestamps) give exactly the tokens of kw_dec_linear + kw_greedy_step -- also when rows finish
    early on EOS (pad after it, the stop count) -- and the fused launch really ran (lm_greedy_last)."""
    g = torch.Generator(device="cuda").manual_seed(9)
    feats = torch.randn(6, TINY.num_mel_bins, TINY.n_frames, device="cuda", generator=g) * 0.5
    gen = generation_constants(TINY)
    if eos is not None:
        gen.eos_token_id = eos
    kw = dict(language="ja", task="transcribe", return_timestamps=False, max_length=40, generation_config=gen)
    eng = tiny16.engine
    out = {}
    try:
        for fuse in (False, True):
            eng.fuse_lm_greedy = fuse
            out[fuse] = tiny16.generate(feats, **kw).cpu()
            assert tiny16._sessions[(6, 1)].lm_greedy_last == fuse
    finally:
        eng.fuse_lm_greedy = True
    assert torch.equal(out[False], out[True])


@pytest.mark.parametrize("k", [1, 2, 3])
def test_stop_check_fires_after_last_eos(tiny16, k):
    """The host stop check reads the unfinished-row count a few replays behind, from a pinned slot that first gets
    a -1 sentinel (r03al).  A slot read before its copy lands would never stop the loop (silently decoding to
    max_length): once every row has emitted EOS the loop must stop within its lag (check_every steps) plus one
    replay.  EOS is chosen from a first run as a token every row emits, so every row finishes early."""
    g = torch.Generator(device="cuda").manual_seed(13)
    feats = torch.randn(6, TINY.num_mel_bins, TINY.n_frames, device="cuda", generator=g) * 0.5
    gen = generation_constants(TINY)
    kw = dict(language="ja", task="transcribe", return_timestamps=False, max_length=120)
    eng = tiny16.engine
    try:
        eng.steps_per_replay = k
        ids = tiny16.generate(feats, generation_config=gen, **kw).cpu()
        P = 4 if int(ids[0, 0]) == gen.decoder_start_token_id else 0  # (prompt kept in the output or not)
        body = ids[:, P:]
        first = {}  # token -> the latest step at which a row first emits it
        for t in set(body[0].tolist()):
            hits = [(row == t).nonzero() for row in body]
            if all(len(h) for h in hits):
                first[t] = max(int(h[0]) for h in hits)
        if not first:
            pytest.skip("no token common to every row")
        # prefer an EOS every row reaches after a few steps (the stop then fires mid-loop, not right after prefill)
        late = {t: v for t, v in first.items() if v >= 4}
        eos, s = min((late or first).items(), key=lambda kv: kv[1])
        if s + 1 + 4 + k >= 120 - P:
            pytest.skip("rows finish too close to max_length")
        gen2 = generation_constants(TINY)
        gen2.eos_token_id = eos
        out = tiny16.generate(feats, generation_config=gen2, **kw).cpu()
        steps = tiny16._session(6).last_steps
    finally:
        eng.steps_per_replay = 2
    print(f"k {k}: P {P} eos {eos} last EOS at body index {s}; out {tuple(out.shape)}; steps issued {steps}")
    assert out.shape[1] == P + s, (out.shape, P, s)  # the last row's EOS ends its segment and is stripped (HF)
    # the loop issued at most the steps up to the last EOS, the lag (4 steps) and one more replay
    assert s + 1 <= steps <= s + 1 + 4 + k, (steps, s, k)


@pytest.mark.parametrize("block", ["kw_dec_qkv_self", "kw_dec_xq_cross"])
def test_handoff_timeout_raises(gold, tiny16, block):
    """A fused decode block whose in-launch hand-off times out must fail the call, not return tokens (VERDICT r3
    item 3; SURVEY §8b "HIP errors -> RuntimeError"): the workspace's fault-injection word makes ONE launch's
    first projection workgroup skip its publish, that launch's consumers time out (NaN rows + status word), and
    generate() raises KWError after its final synchronize.  The session re-arms its workspaces, so the next
    call returns the tokens of an undisturbed run."""
    from kwhisper._lib import KWError

    g = gold("tiny_fp32")
    feats = torch.from_numpy(oracle_features(TINY, g["cases"][:2])).cuda()
    kw = dict(language="ja", task="transcribe", max_length=24)
    want = tiny16.generate(feats, **kw).cpu().numpy()
    sess = tiny16._session(2)
    words = {name: (ws, off) for name, ws, off in sess.status_words()}
    assert {"kw_dec_qkv_self", "kw_dec_xq_cross"} <= set(words)  # the greedy bf16 step runs both fused blocks
    ws, off = words[block]
    ws.view(torch.int32)[off // 4 + 1] = 1  # arm the fault-injection word
    with pytest.raises(KWError, match=block):
        tiny16.generate(feats, **kw)
    assert int(ws.view(torch.int32)[off // 4 + 1]) == 0  # consumed by exactly one launch
    assert all(int(w.view(torch.int32)[o // 4]) == 0 for _, w, o in sess.status_words())  # re-armed
    np.testing.assert_array_equal(tiny16.generate(feats, **kw).cpu().numpy(), want)


def test_own_streams_recycled():
    """kwhisper._lib.new_stream (the HIP streams of their own that captures, prefill parts, encoder parts and lanes
    use) hands a stream back out once its owner is garbage collected or it is released, instead of making more:
    repeated sessions / lane calls do not grow the process's streams."""
    import gc

    from kwhisper import _lib as L

    class Owner:
        pass

    n0 = len(L._OWN_STREAMS)
    for _ in range(5):
        o = Owner()
        L.new_stream(owner=o)
        del o
        gc.collect()
    assert len(L._OWN_STREAMS) <= n0 + 1
    s1 = L.new_stream()
    L.release_stream(s1)
    assert L.new_stream() is s1
    L.release_stream(s1)
