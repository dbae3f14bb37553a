"""The BASELINE workloads themselves on the GPU, against fixtures of the reference path.

* config 3 (the bench workload: large-v3, 32 clips, greedy, 128 new tokens, no timestamps;
  run_pseudo_labelling.py:338): the bf16 production path -- graph-replayed generate(), packed
  LayerNorm-folded decode linears, LM head kernel -- against transformers' fp32 run of the same 32 clips
  (tests/golden/large_v3_b32_fp32.npz): margin-gated token equality, teacher-forced max / mean logit error,
  batch invariance; and the fp32 parity mode bit-exact at the same size.
* config 5 (kotoba-whisper-v2.0 layout, beam 5 + timestamps, chunked pipeline; run_short_form_eval.py:184-191):
  fp32 beam search bit-exact, bf16 beam hypotheses rescored by the fp32 engine, and the chunked
  ASRPipeline against the real transformers pipeline's output.
* config 4 (run_pseudo_labelling.py:333-344 with timestamps, its default :99-102): pseudo_label() over the
  bf16 large-v3 engine -- the config's own teacher -- at batch 32 over the ReazonSpeech-length stand-in clips,
  against transformers' fp32 run of the same clips (tests/golden/large_v3_ts_b32_fp32.npz): the fp32 mode
  bit-exact, the bf16 path margin-gated; W = 2 (two spawned processes on cuda:0 over gloo) gathers the W = 1
  predictions in dataset order.  The tiny engine's loop tests (resume, legacy layout) stay beside it.

Every measured error is printed (run with -s; the round's pytest log is committed under profiles/).
"""
import json
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from kwhisper.config import KOTOBA_V2, LARGE_V3, TINY, generation_constants  # noqa: E402
from kwhisper.synthetic import synthetic_state_dict  # noqa: E402

from _util import OracleFeatureExtractor, StubTok, clip_audio, jsonable, oracle_features  # noqa: E402

# bf16 noise floor for greedy tokens: a step whose fp32 top-1/top-2 margin is below this may flip under bf16
# arithmetic.  A flip needs both logits to move, so the floor is 2x the engine's measured max teacher-forced
# logit error at config 3 (0.097, r02k); the reference's own bf16 model errs up to 0.19 and its greedy tokens
# leave the fp32 ones at steps whose margin is as low as 0.024 (tests/golden/large_v3_bf16ref.npz).
MARGIN_FLOOR = 0.2


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _model(shape, dtype, pad=None, seed=0):
    from kwhisper.generation import KWhisperForConditionalGeneration

    return KWhisperForConditionalGeneration.from_state_dict(
        shape, synthetic_state_dict(shape, seed), dtype=dtype, generation_config=generation_constants(shape, pad))


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _gated_equal(toks, want, margin, floor=MARGIN_FLOOR):
    """Rows equal up to each row's first step whose reference margin is below ``floor``; returns the
    number of tokens compared."""
    n = 0
    for b in range(want.shape[0]):
        unsafe = np.nonzero(margin[b] < floor)[0]
        upto = int(unsafe[0]) if unsafe.size else want.shape[1]
        np.testing.assert_array_equal(toks[b, :upto], want[b, :upto], err_msg=f"row {b} (first unsafe step {upto})")
        n += upto
    return n


# ---------------------------------------------------------------------------------------------------------
# config 3


@pytest.fixture(scope="module")
def large_b32_gold(gold):
    g = gold("large_v3_b32_fp32")
    return g, oracle_features(LARGE_V3, g["cases"])


def test_config3_bf16_generate_b32(gold, large_b32_gold):
    """The measured bf16 path at the bench's exact shape: B = 32, 128 graph-replayed decode steps.

    Tolerances are the REFERENCE's own bf16 noise (tests/golden/large_v3_bf16ref.npz: the same HF model cast to
    bf16, as run_pseudo_labelling.py:229,338 runs it, on all 32 clips): the engine's encoder and teacher-forced
    logits must be at least as close to fp32 as the reference's bf16 model is (x1.25 for the encoder, whose
    bf16 rounding points differ), and its greedy tokens must leave the fp32 tokens no earlier on average, and
    agree with them at no fewer positions, than the reference bf16 model's own greedy tokens do."""
    g, feats_np = large_b32_gold
    r = gold("large_v3_bf16ref")
    rows = [int(x) for x in r["rows"]]
    model = _model(LARGE_V3, torch.bfloat16)
    feats = torch.from_numpy(feats_np).cuda()
    eng = model.engine
    # encoder (bf16 residual stream, as the reference's bf16 model)
    enc = eng.encode(feats)
    e = enc.view(32, 1500, 1280).float().cpu().numpy()[:, ::250, :]
    ref = g["enc_slice"]

    def enc_err(x, y):
        return np.abs(x - y).max() / np.abs(y).max(), np.abs(x - y).mean() / np.abs(y).mean()

    ours_all, ours, theirs = enc_err(e, ref), enc_err(e[rows], ref[rows]), enc_err(r["enc_slice"], ref[rows])
    print(f"\nconfig3 bf16 encoder vs fp32 reference (max|err|/max|ref|, mean|err|/mean|ref|): all 32 rows "
          f"{ours_all[0]:.4f} / {ours_all[1]:.4f}; rows {rows}: engine {ours[0]:.4f} / {ours[1]:.4f}, "
          f"reference bf16 model {theirs[0]:.4f} / {theirs[1]:.4f}")
    assert ours[0] <= 1.25 * theirs[0] and ours[1] <= 1.25 * theirs[1]
    assert ours_all[0] < 0.05 and ours_all[1] < 0.02
    # teacher-forced logits through the production decode kernels (packed weights, folded LayerNorms, LM head)
    sess = eng.new_session(32, enc)
    seq = torch.from_numpy(g["greedy_sequences"])
    lg = sess.teacher_forced_logits(seq[:, :-1], 4)
    idx = torch.from_numpy(g["greedy_logits_top_idx"].astype(np.int64)).cuda()
    got = torch.gather(lg[:, : idx.shape[1]], -1, idx).cpu().numpy()
    err = np.abs(got - g["greedy_logits_top_val"])
    top1 = lg[:, : idx.shape[1]].argmax(-1).cpu().numpy()
    agree = (top1 == g["greedy_logits_top_idx"][..., 0]).mean()
    ref_err = np.abs(r["tf_logits_at_fp32_top8"] - g["greedy_logits_top_val"][rows])
    print(f"config3 bf16 teacher-forced top-8 logit err over {err.size} values: max {err.max():.4f} "
          f"mean {err.mean():.5f} p99 {np.percentile(err, 99):.4f}; top-1 agreement {agree:.4f}; on rows {rows}: "
          f"engine max {err[rows].max():.4f} mean {err[rows].mean():.5f}, reference bf16 model max "
          f"{ref_err.max():.4f} mean {ref_err.mean():.5f}")
    assert err[rows].max() <= ref_err.max() and err[rows].mean() <= ref_err.mean()
    assert err.max() < 0.2 and err.mean() < 0.03
    # teacher-forced greedy choice at EVERY step the fp32 reference decides by a margin >= MARGIN_FLOOR (the fed
    # sequence keeps the engine on the reference trajectory past any earlier low-margin step): the processed
    # argmax (SuppressTokens, SuppressTokensAtBegin at the first step; logits_process.py:1816-1906) equals the
    # fp32 reference's token
    gen = generation_constants(LARGE_V3)
    n_pos = g["greedy_margin"].shape[1]
    proc = lg[:, :n_pos].clone()
    proc[:, :, torch.tensor(gen.suppress_tokens, device=proc.device)] = -float("inf")
    proc[:, 0, torch.tensor(gen.begin_suppress_tokens, device=proc.device)] = -float("inf")
    choice = proc.argmax(-1).cpu().numpy()
    want_tok = g["greedy_sequences"][:, 4: 4 + n_pos]
    safe = g["greedy_margin"] >= MARGIN_FLOOR
    bad = np.argwhere(safe & (choice != want_tok))
    print(f"config3 bf16 teacher-forced greedy choice: {int(safe.sum())} of {safe.size} steps with fp32 margin >= "
          f"{MARGIN_FLOOR} compared, {len(bad)} differ; all steps agree at {(choice == want_tok).mean():.4f}")
    assert len(bad) == 0, f"(row, step) pairs whose safe-margin greedy choice differs: {bad[:8].tolist()}"
    del lg, proc, sess
    _free()
    # the graph-replayed generate() (what bench.py times)
    toks = model.generate(feats, language="ja", task="transcribe", max_length=128).cpu().numpy()
    want = g["greedy_tokens"]
    assert toks.shape == want.shape
    n = _gated_equal(toks, want, g["greedy_margin"])
    full = int((toks == want).all(1).sum())

    def first_div(t):
        return np.array([int(np.nonzero(t[b] != want[b])[0][0]) if (t[b] != want[b]).any() else want.shape[1]
                         for b in range(want.shape[0])])

    ref_toks = r["greedy_tokens"]
    ours_fd, ref_fd = first_div(toks[rows]), first_div(ref_toks)
    ours_eq, ref_eq = (toks[rows] == want[rows]).mean(), (ref_toks == want[rows]).mean()
    print(f"config3 bf16 generate: {n} of {want.size} tokens compared (margin >= {MARGIN_FLOOR}), all equal; "
          f"{full}/32 rows identical end to end; {(toks == want).mean():.4f} of all positions equal; vs fp32 "
          f"on rows {len(rows)}: first divergence step mean engine {ours_fd.mean():.2f} / reference bf16 model "
          f"{ref_fd.mean():.2f}, equal positions engine {ours_eq:.4f} / reference bf16 model {ref_eq:.4f}, rows "
          f"identical engine {int((ours_fd == want.shape[1]).sum())} / reference bf16 model "
          f"{int((ref_fd == want.shape[1]).sum())}")
    # equal positions: no worse than the reference's own bf16 model.  The mean first-divergence step of 32 greedy
    # trajectories moves by a few steps with any change of summation order at equal teacher-forced error (71.4
    # and 68.3 for two cross-attention kernels whose logit errors are 0.0914 / 0.0229 and 0.0899 / 0.0230, HF
    # bf16 71.0): held within 5 % of the reference bf16 model's (the per-step check above is the strict one)
    assert ours_eq >= ref_eq and ours_fd.mean() >= 0.95 * ref_fd.mean()
    # batch invariance: two of the clips alone give the rows they get inside the batch of 32
    sub = [0, 17]
    toks2 = model.generate(feats[sub], language="ja", task="transcribe", max_length=128).cpu().numpy()
    np.testing.assert_array_equal(toks2, toks[sub])
    del model
    _free()


def test_config3_fp32_generate_b32_bitexact(large_b32_gold):
    """North star: greedy token ids bit-exact with the HF fp32 reference, at the config-3 shape (fp32 parity
    mode: exact-fp32 MFMA GEMMs, separate LayerNorms)."""
    g, feats_np = large_b32_gold
    model = _model(LARGE_V3, torch.float32)
    feats = torch.from_numpy(feats_np).cuda()
    toks = model.generate(feats, language="ja", task="transcribe", max_length=128)
    np.testing.assert_array_equal(toks.cpu().numpy(), g["greedy_tokens"])
    # north star: logits within 1e-3 of the HF fp32 reference -- teacher-forced along transformers' own greedy
    # sequence, at its top-8 ids of every one of the 124 steps of all 32 rows (raw logits, utils.py:2894)
    eng = model.engine
    sess = eng.new_session(32, eng.encode(feats))
    lg = sess.teacher_forced_logits(torch.from_numpy(g["greedy_sequences"])[:, :-1], 4)
    idx = torch.from_numpy(g["greedy_logits_top_idx"].astype(np.int64)).cuda()
    got = torch.gather(lg[:, : idx.shape[1]], -1, idx).cpu().numpy()
    err = np.abs(got - g["greedy_logits_top_val"])
    print(f"\nconfig3 fp32 teacher-forced logits vs HF fp32 over {err.size} values: max {err.max():.2e} mean "
          f"{err.mean():.2e} (|logit| max {np.abs(g['greedy_logits_top_val']).max():.2f})")
    np.testing.assert_allclose(got, g["greedy_logits_top_val"], atol=1e-3, rtol=0)
    del model, sess, lg
    _free()


# ---------------------------------------------------------------------------------------------------------
# config 5


@pytest.fixture(scope="module")
def kotoba32():
    m = _model(KOTOBA_V2, torch.float32)
    yield m
    del m
    _free()


@pytest.mark.parametrize("mode", ["beam5_ts", "beam5"])
def test_config5_kotoba_fp32_beam_bitexact(gold, kotoba32, mode):
    g = gold("kotoba_v2_beam_fp32")
    kw = {"beam5_ts": dict(return_timestamps=True), "beam5": dict(return_timestamps=False)}[mode]
    feats = torch.from_numpy(oracle_features(KOTOBA_V2, g["cases"])).cuda()
    toks = kotoba32.generate(feats, language="ja", task="transcribe", num_beams=5, max_length=48, **kw)
    np.testing.assert_array_equal(toks.cpu().numpy(), g[f"{mode}_tokens"])


def _tf_logprobs(eng, enc_row, seq, P):
    """Per-token log-softmax of the teacher-forced logits of ``seq`` (1-D, prompt + generated) for positions
    P..len-1 (the generated tokens)."""
    sess = eng.new_session(1, enc_row)
    t = torch.as_tensor(seq, dtype=torch.int64)[None]
    lg = sess.teacher_forced_logits(t, P)[0, : t.shape[1] - P].float()
    lp = torch.log_softmax(lg, -1)
    return lp.gather(-1, t[0, P:].cuda()[:, None])[:, 0].double().cpu().numpy()


def test_config5_kotoba_bf16_beam_rescored(gold, kotoba32):
    """bf16 beam search (no timestamps, one seek pass) on the kotoba-v2.0 layout: every item's chosen
    hypothesis, rescored by the fp32 engine (pinned bit-exact to HF above), is as good as the fp32 beam's
    choice within the bf16 scoring noise of the two hypotheses (HF beam score: sum of log-probs / length,
    utils.py:3182)."""
    g = gold("kotoba_v2_beam_fp32")
    gen = generation_constants(KOTOBA_V2)
    feats = torch.from_numpy(oracle_features(KOTOBA_V2, g["cases"])).cuda()
    m16 = _model(KOTOBA_V2, torch.bfloat16)
    kw = dict(language="ja", task="transcribe", num_beams=5, max_length=48, return_timestamps=False)
    t16 = m16.generate(feats, **kw).cpu().numpy()
    t32 = g["beam5_tokens"]
    prompt = [gen.decoder_start_token_id, gen.lang_to_id["<|ja|>"], gen.task_to_id["transcribe"],
              gen.no_timestamps_token_id]
    P, max_new = len(prompt), 48  # max_length grows by the prompt (generation_whisper.py:1935-1940)
    e32 = kotoba32.engine.encode(feats).view(4, 1500, -1)
    e16 = m16.engine.encode(feats).view(4, 1500, -1)

    def hyp(row):
        r = [int(x) for x in row]
        while r and r[-1] == gen.pad_token_id:
            r.pop()
        return prompt + r + ([gen.eos_token_id] if len(r) < max_new else [])

    same = 0
    for b in range(4):
        h16, h32 = hyp(t16[b]), hyp(t32[b])
        s = {}
        for name, h in (("h16", h16), ("h32", h32)):
            lp32 = _tf_logprobs(kotoba32.engine, e32[b:b + 1].reshape(1500, -1), h, P)
            lp16 = _tf_logprobs(m16.engine, e16[b:b + 1].reshape(1500, -1), h, P)
            s[name] = (lp32.sum() / len(lp32), lp16.sum() / len(lp16))
        tol = abs(s["h16"][1] - s["h16"][0]) + abs(s["h32"][1] - s["h32"][0]) + 1e-4
        same += h16 == h32
        print(f"\nconfig5 bf16 beam item {b}: same hypothesis {h16 == h32}; fp32 score of bf16 choice "
              f"{s['h16'][0]:.5f} vs fp32 choice {s['h32'][0]:.5f} (tolerance {tol:.5f})")
        assert s["h16"][0] >= s["h32"][0] - tol
    print(f"config5 bf16 beam: {same}/4 items chose the fp32 hypothesis")
    del m16
    _free()


@pytest.mark.parametrize("fe_kind", ["oracle", "hip"])
def test_config5_pipeline_kotoba_fp32(gold, kotoba32, fe_kind):
    """run_short_form_eval.py:184-191 at config 5: ASRPipeline(chunk_length_s=15, batch_size=4, beam 5,
    timestamps) == the real transformers pipeline (tests/golden/pipeline_kotoba_v2_fp32.npz), window batch by
    window batch and in the merged text / chunks.  ``fe_kind``: the oracle log-mel (exact inputs) or the
    product HIP log-mel."""
    from kwhisper.pipeline import ASRPipeline

    g = gold("pipeline_kotoba_v2_fp32")
    _check_pipeline(g, kotoba32, KOTOBA_V2, fe_kind)


def _check_pipeline(g, model, shape, fe_kind, batch_size=None, ts_keys=None):
    from kwhisper.pipeline import ASRPipeline

    gk = json.loads(str(g["generate_kwargs"]))
    fe = OracleFeatureExtractor(shape.num_mel_bins) if fe_kind == "oracle" else None
    pipe = ASRPipeline(model, feature_extractor=fe, tokenizer=StubTok(generation_constants(shape)),
                       chunk_length_s=float(g["chunk_length_s"]), batch_size=batch_size or int(g["batch_size"]),
                       generate_kwargs=gk)
    calls = []
    orig = model.generate

    def rec(*a, **kw):
        out = orig(*a, **kw)
        calls.append((out["sequences"] if isinstance(out, dict) else out).cpu().numpy())
        return out

    model.generate = rec
    try:
        for key in ts_keys or [k[:-7] for k in g if k.endswith("_result")]:
            ts = key == "ts1"
            calls.clear()
            got = pipe([{"array": clip_audio(c), "sampling_rate": 16000} for c in g["clips"]], return_timestamps=ts)
            if batch_size is None:  # the reference's window batches, one by one
                assert len(calls) == int(g[f"{key}_n_calls"])
                for i, c in enumerate(calls):
                    np.testing.assert_array_equal(c, g[f"{key}_call{i}"], err_msg=f"{key} window batch {i}")
            assert jsonable(got) == json.loads(str(g[f"{key}_result"]))
    finally:
        del model.generate


def test_config5_pipeline_kotoba_bf16_runs(gold):
    """The same pipeline on the bf16 engine (the measured configuration) over device beam search: the merged text
    equals the real transformers fp32 pipeline's on this fixture (measured r03: both clips, every character; the
    engine is deterministic, so this holds run to run).  A kernel change that flips a beam choice here fails the
    test and is triaged with test_config5_kotoba_bf16_beam_rescored, which bounds a bf16 choice's quality by
    fp32 rescoring rather than by identity."""
    from kwhisper.pipeline import ASRPipeline

    g = gold("pipeline_kotoba_v2_fp32")
    m16 = _model(KOTOBA_V2, torch.bfloat16)
    gk = json.loads(str(g["generate_kwargs"]))
    pipe = ASRPipeline(m16, tokenizer=StubTok(generation_constants(KOTOBA_V2)), chunk_length_s=15,
                       batch_size=int(g["batch_size"]), generate_kwargs=gk)
    got = pipe([{"array": clip_audio(c), "sampling_rate": 16000} for c in g["clips"]], return_timestamps=True)
    want = json.loads(str(g["ts1_result"]))
    for i, (a, b) in enumerate(zip(jsonable(got), want)):
        ta, tb = a["text"], b["text"]
        k = next((j for j in range(min(len(ta), len(tb))) if ta[j] != tb[j]), min(len(ta), len(tb)))
        print(f"\nconfig5 bf16 pipeline clip {i}: text identical {ta == tb}; common prefix {k} of {len(tb)} chars; "
              f"{len(a['chunks'])} vs {len(b['chunks'])} chunks")
        assert len(ta) > 0 and all(set(c) == {"timestamp", "text"} for c in a["chunks"])
        assert ta == tb, f"clip {i}: bf16 pipeline text differs from the fp32 reference after {k} chars"
    del m16
    _free()


def test_config5_pipeline_lanes_equal_one_lane(gold):
    """ASRPipeline(lanes=2) on the bf16 kotoba-v2 engine (beam 5 + timestamps, window batches of 2 so that lanes
    overlap): two window batches decode at once on model.lane() handles from two host threads, each on its own
    stream; the merged output is identical to the one-lane run's (every beam graph per lane, stream-local syncs)."""
    from kwhisper.pipeline import ASRPipeline

    g = gold("pipeline_kotoba_v2_fp32")
    m16 = _model(KOTOBA_V2, torch.bfloat16)
    gk = json.loads(str(g["generate_kwargs"]))
    clips = [{"array": clip_audio(c), "sampling_rate": 16000} for c in g["clips"]] * 2
    out = {}
    for lanes in (1, 2):
        pipe = ASRPipeline(m16, tokenizer=StubTok(generation_constants(KOTOBA_V2)), chunk_length_s=15, batch_size=2,
                           generate_kwargs=gk, lanes=lanes)
        out[lanes] = jsonable(pipe(clips, return_timestamps=True))
    print(f"\nconfig5 pipeline lanes: {len(clips)} clips, outputs equal {out[1] == out[2]}")
    assert out[1] == out[2]
    del m16
    _free()


@pytest.fixture(scope="module")
def c5_b64(gold, kotoba32):
    """Config 5 at its BASELINE batch through ASRPipeline on the fp32 engine: 22 of tools/bench_configs.py's 30 s
    clips -> 66 windows -> window batches of 64 and 2 (bs = 64 windows x 5 beams = 320 rows; run_short_form_eval.py:
    110-117,184-191, chunk_length_s 15, timestamps).  Returns the fixture, the pipeline output and every
    generate() call (features, kwargs, tokens)."""
    from kwhisper.pipeline import ASRPipeline

    g = gold("pipeline_kotoba_v2_b64_fp32")
    gk = json.loads(str(g["generate_kwargs"]))
    pipe = ASRPipeline(kotoba32, feature_extractor=OracleFeatureExtractor(KOTOBA_V2.num_mel_bins),
                       tokenizer=StubTok(generation_constants(KOTOBA_V2)), chunk_length_s=float(g["chunk_length_s"]),
                       batch_size=int(g["batch_size"]), generate_kwargs=gk)
    calls = []
    orig = kotoba32.generate

    def rec(feats, **kw):
        out = orig(feats, **kw)
        calls.append((feats, kw, (out["sequences"] if isinstance(out, dict) else out).cpu().numpy()))
        return out

    kotoba32.generate = rec
    try:
        got = pipe([{"array": clip_audio(c), "sampling_rate": 16000} for c in g["clips"]], return_timestamps=True)
    finally:
        del kotoba32.generate
    return g, gk, got, calls


def test_config5_b64_pipeline_fp32_bitexact(c5_b64):
    """The fp32 engine at R = 320 beam rows: every window batch's tokens and the merged text of the 22 clips equal
    the real transformers fp32 pipeline's (tests/golden/pipeline_kotoba_v2_b64_fp32.npz)."""
    g, gk, got, calls = c5_b64
    assert len(calls) == int(g["ts1_n_calls"]) == 2 and calls[0][0].shape[0] == 64
    for i, (_, _, toks) in enumerate(calls):
        np.testing.assert_array_equal(toks, g[f"ts1_call{i}"], err_msg=f"window batch {i}")
    assert jsonable(got) == json.loads(str(g["ts1_result"]))
    print(f"\nconfig5 b64: fp32 engine bit-exact with transformers at 64 windows x 5 beams (2 window batches, "
          f"{len(got)} clips' merged text)")


def test_config5_b64_bf16_beam_vs_reference_bf16(gold, kotoba32, c5_b64):
    """The bf16 engine on the 64-window batch (320 beam rows) against the REFERENCE's own bf16 beam search on the
    same windows (tests/golden/pipeline_kotoba_v2_b64_bf16.npz: transformers' pipeline with the model in bfloat16,
    as run_short_form_eval.py runs it).  Over 128 beam steps a bf16 score perturbation can prune the fp32 beam's
    eventual winner early (path dependence), so the bar is the reference's own: every chosen hypothesis is rescored
    by the fp32 engine (bit-exact with transformers; HF beam score = sum of log-probs / length, utils.py:3182) and
    the engine's mean fp32-score deficit to the fp32 choice, and its number of windows off the fp32 choice beyond the
    two hypotheses' bf16 scoring noise, are no worse than the reference bf16 model's (x1.25 + 1e-3 on the mean)."""
    g, gk, _, calls = c5_b64
    r = gold("pipeline_kotoba_v2_b64_bf16")
    gen = generation_constants(KOTOBA_V2)
    feats, kw, t32 = calls[0]
    m16 = _model(KOTOBA_V2, torch.bfloat16)
    t16 = m16.generate(feats, **kw).cpu().numpy()
    tref = r["ts1_call0"]
    prompt = [gen.decoder_start_token_id, gen.lang_to_id["<|ja|>"], gen.task_to_id["transcribe"]]  # timestamps
    P, max_new = len(prompt), int(gk["max_length"])
    e32 = kotoba32.engine.encode(feats).view(64, 1500, -1)
    e16 = m16.engine.encode(feats).view(64, 1500, -1)

    def hyp(row):
        x = [int(t) for t in row]
        while x and x[-1] == gen.pad_token_id:
            x.pop()
        return prompt + x + ([gen.eos_token_id] if len(x) < max_new else [])

    cache = {}

    def score(eng, e, b, h, tag):
        key = (tag, b, tuple(h))
        if key not in cache:
            lp = _tf_logprobs(eng, e[b:b + 1].reshape(1500, -1), h, P)
            cache[key] = lp.sum() / len(lp)
        return cache[key]

    stats = {}
    for name, toks in (("engine", t16), ("reference bf16", tref)):
        deficits, off = [], 0
        for b in range(64):
            h, h32 = hyp(toks[b]), hyp(t32[b])
            if h == h32:
                deficits.append(0.0)
                continue
            s_h, s_32 = score(kotoba32.engine, e32, b, h, "f32"), score(kotoba32.engine, e32, b, h32, "f32")
            n_h, n_32 = score(m16.engine, e16, b, h, "b16"), score(m16.engine, e16, b, h32, "b16")
            tol = abs(n_h - s_h) + abs(n_32 - s_32) + 1e-4
            deficits.append(max(0.0, s_32 - s_h))
            off += int(s_h < s_32 - tol)
        same = sum(1 for b in range(64) if hyp(toks[b]) == hyp(t32[b]))
        stats[name] = (same, float(np.mean(deficits)), float(np.max(deficits)), off)
    for name, (same, mean_d, max_d, off) in stats.items():
        print(f"\nconfig5 b64 {name}: {same}/64 windows chose the fp32 hypothesis; fp32-score deficit mean {mean_d:.5f} "
              f"max {max_d:.5f}; {off} windows beyond the bf16 scoring noise")
    eng, ref = stats["engine"], stats["reference bf16"]
    assert eng[1] <= 1.25 * ref[1] + 1e-3 and eng[3] <= max(ref[3], 1) * 1.25
    del m16
    _free()


# ---------------------------------------------------------------------------------------------------------
# tiny pipeline fixtures (the reference's own pipeline; no transformers on the GPU box)


@pytest.fixture(scope="module")
def tiny32():
    m = _model(TINY, torch.float32)
    yield m
    del m


@pytest.mark.parametrize("fe_kind", ["oracle", "hip"])
def test_pipeline_chunked_tiny_vs_reference(gold, tiny32, fe_kind):
    """ASRPipeline(chunk_length_s=15, batch_size=3) on a 40 s and a 7 s clip, with and without timestamps,
    == transformers' pipeline (tests/golden/pipeline_tiny_fp32.npz)."""
    _check_pipeline(gold("pipeline_tiny_fp32"), tiny32, TINY, fe_kind)


def test_pipeline_longform_tiny_vs_reference(gold, tiny32):
    """ASRPipeline without chunking on 45 / 70 / 12 s clips: each item one long-form generate (the seek
    loop; the pipeline's default beam 5) == transformers' pipeline at batch_size 1
    (tests/golden/pipeline_tiny_longform_fp32.npz)."""
    _check_pipeline(gold("pipeline_tiny_longform_fp32"), tiny32, TINY, "oracle")


def test_pipeline_longform_tiny_batched(gold, tiny32):
    """The same clips at batch_size 3 (transformers 5.15 cannot collate long-form items of different lengths,
    pipelines/base.py:118, so this batch has no reference): the two > 30 s clips, which take the long-form
    path either way, give the batch-1 reference's output; the 12 s clip, which batched becomes a masked
    long-form item instead of one 30 s window, only has to run."""
    from kwhisper.pipeline import ASRPipeline

    g = gold("pipeline_tiny_longform_fp32")
    gk = json.loads(str(g["generate_kwargs"]))
    pipe = ASRPipeline(tiny32, feature_extractor=OracleFeatureExtractor(TINY.num_mel_bins),
                       tokenizer=StubTok(generation_constants(TINY)), batch_size=3, generate_kwargs=gk)
    got = jsonable(pipe([{"array": clip_audio(c), "sampling_rate": 16000} for c in g["clips"]], return_timestamps=True))
    want = json.loads(str(g["ts1_result"]))
    long_items = [i for i, c in enumerate(g["clips"]) if float(str(c).split(":")[2]) > 30]
    assert long_items == [0, 1]
    for i in long_items:
        assert got[i] == want[i], i
    assert len(got[2]["text"]) > 0


# ---------------------------------------------------------------------------------------------------------
# config 4: the pseudo-labelling loop over the engine

C4_KW = dict(language="ja", task="transcribe", return_timestamps=True, max_length=128)  # :99-102, max_label_length


def _c4_features(g):
    """Log-mel (oracle, f64 STFT) of the fixture's config-4 stand-in clips zero-padded to 30 s, as the feature
    extractor pads them (feature_extraction_whisper.py:300-307).  Clip i of the stand-in is
    reazon_audio(i, duration); the fixture names its clips by ``clip_ids`` (the first 32 when absent)."""
    from kwhisper.synthetic import reazon_audio
    from oracle.mel import log_mel, pad_or_trim

    ids = g["clip_ids"] if "clip_ids" in g else np.arange(len(g["durations"]))
    clips = [pad_or_trim(reazon_audio(int(i), float(d))) for i, d in zip(ids, g["durations"])]
    return torch.from_numpy(log_mel(np.stack(clips), LARGE_V3.num_mel_bins)).cuda()


# the first 32 stand-in clips (every row one seek pass on the oracle log-mel: no stand-in clip takes a second pass
# under transformers' fp32 large-v3 there, profiles/r04d_multipass_scan.json).  The multi-pass case on the product's
# own HIP log-mel is pinned by test_config4_hipmel_multipass (tests/golden/large_v3_c4_hipmel.npz).
C4_FIXTURES = ["large_v3_ts_b32_fp32"]


@pytest.fixture(scope="module", params=C4_FIXTURES)
def c4_gold(gold, request):
    g = gold(request.param)
    return request.param, g, _c4_features(g)


def _c4_pseudo_label(model, durations, feats_all, batch_size):
    from kwhisper.pseudo_label import pseudo_label

    n = len(durations)
    pad = model.generation_config.eos_token_id  # the tokenizer's pad id (<|endoftext|>), run_pseudo_labelling.py:339
    return pseudo_label(model, lambda idx: feats_all[list(idx)], n, batch_size=batch_size, gen_kwargs=C4_KW,
                        pad_token_id=pad, comm_device="cpu")


def test_config4_fp32_pseudo_label_bitexact(c4_gold):
    """Config 4 at its own teacher in the fp32 parity mode: pseudo_label() (W = 1, batch 32) over large-v3 with
    timestamps returns transformers' fp32 tokens exactly, row for row (the split timestamp sampler at
    V = 51866, B = 32, and the seek loop over zero-padded short clips).  On the multi-pass fixture >= 8 rows take
    a second seek pass (a re-encode of the shifted mel, generation_whisper.py:785-903, with the cumulative
    max_length growth :1935-1940), and the engine's per-row pass counts equal transformers'."""
    name, g, feats = c4_gold
    model = _model(LARGE_V3, torch.float32)
    ids, preds = _c4_pseudo_label(model, g["durations"], feats, 32)
    assert ids == list(range(32))
    np.testing.assert_array_equal(np.stack(preds), g["tokens"])
    assert model.stats["passes"] == int(g["passes"].max())
    np.testing.assert_array_equal(model.stats["row_passes"], g["passes"])
    del model
    _free()


def _c4_worker(rank, world, port, out_dir, batch_size, name):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", f"{name}.npz")))
        model = _model(LARGE_V3, torch.bfloat16)
        feats = _c4_features(g)
        ids, preds = _c4_pseudo_label(model, g["durations"], feats, batch_size)
        np.savez(os.path.join(out_dir, f"c4_r{rank}.npz"), ids=np.array(ids), preds=np.stack(preds))
    finally:
        dist.destroy_process_group()


def test_config4_bf16_pseudo_label_w1_w2(c4_gold, tmp_path):
    """Config 4 as measured: the bf16 large-v3 engine in the reference's loop (run_pseudo_labelling.py:333-344).
    W = 1 at batch 32: tokens equal transformers' fp32 run up to each row's first step whose fp32 top-1 / top-2
    margin is below MARGIN_FLOOR.  W = 2 (two processes on cuda:0, gloo, batch 16 each: rank r takes batch r,
    accelerate's BatchSamplerShard) gathers exactly the W = 1 predictions in dataset order (the decode is
    batch-invariant: each row's arithmetic does not depend on its batch)."""
    import torch.multiprocessing as mp

    name, g, feats = c4_gold
    model = _model(LARGE_V3, torch.bfloat16)
    ids1, preds1 = _c4_pseudo_label(model, g["durations"], feats, 32)
    assert ids1 == list(range(32))
    toks = np.stack(preds1)
    want = g["tokens"]
    assert toks.shape == want.shape
    n = _gated_equal(toks, want, g["margin"])
    print(f"\nconfig4 bf16 pseudo_label ({name}: large-v3, B = 32, timestamps): {n} of {want.size} tokens compared "
          f"(margin >= {MARGIN_FLOOR}), all equal; {int((toks == want).all(1).sum())}/32 rows identical; "
          f"{(toks == want).mean():.4f} of positions equal; seek passes {model.stats['passes']} (per row "
          f"{model.stats['row_passes'].tolist()}, reference {g['passes'].tolist()})")
    del model
    _free()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_c4_worker, args=(2, port, str(tmp_path), 16, name), nprocs=2, join=True)
    for r in range(2):
        z = np.load(tmp_path / f"c4_r{r}.npz")
        assert z["ids"].tolist() == list(range(32))
        np.testing.assert_array_equal(z["preds"], toks)
    print("config4 bf16 pseudo_label: W=2 (gloo, 2 processes on cuda:0, batch 16 each) == W=1 on 32 items")


def _teacher_forced_per_pass(model, feats, g, floor=MARGIN_FLOOR):
    """The bf16 engine teacher-forced along EVERY seek pass of transformers' fp32 run (the fixture's PassRecorder
    arrays): each pass's segment input is rebuilt from ``feats`` at the recorded seek / frame count (zero-padded to
    3000 frames, generation_whisper.py:1831-1850), encoded by the bf16 engine, and the fp32 pass's sequence is fed
    through the production decode kernels; the processed greedy choice (Suppress -> SuppressAtBegin ->
    WhisperTimeStamp, logits_process.py:1816-2047, applied by the oracle to the engine's logits) must equal the fp32
    token at every step whose fp32 margin is >= ``floor``.  Returns (compared, total, compared in passes >= 2,
    total in passes >= 2, differing (pass entry, step) pairs)."""
    from oracle.generate import process_logits

    gen = generation_constants(LARGE_V3)
    gd = gen.to_dict()
    eng, P = model.engine, 3
    n_cmp = n_tot = n_cmp2 = n_tot2 = 0
    bad = []
    for it in np.unique(g["pass_iter"]):
        ks = np.nonzero(g["pass_iter"] == it)[0]
        seg = torch.zeros((len(ks), feats.shape[1], 3000), device="cuda")
        for i, k in enumerate(ks):
            r, s0, nf = int(g["pass_row"][k]), int(g["pass_seek"][k]), int(g["pass_nframes"][k])
            seg[i, :, :nf] = feats[r, :, s0: s0 + nf]
        L = int(P + g["pass_len"][ks].max())
        seq = g["pass_seq"][ks][:, :L].copy()
        seq[seq < 0] = gen.eos_token_id  # beyond a row's end: any id (causal, never read back)
        sess = eng.new_session(len(ks), eng.encode(seg))
        lg = sess.teacher_forced_logits(torch.from_numpy(seq[:, :-1]), P)
        for i, k in enumerate(ks):
            n = int(g["pass_len"][k])
            rows = lg[i, :n].float().cpu().numpy()
            safe = g["pass_margin"][k, :n] >= floor
            for t in np.nonzero(safe)[0]:
                proc = process_logits(seq[i: i + 1, : P + t], rows[t: t + 1], gd, P, True)
                if int(proc.argmax()) != int(seq[i, P + t]):
                    bad.append((int(k), int(t)))
            n_cmp += int(safe.sum())
            n_tot += n
            if it >= 1:
                n_cmp2 += int(safe.sum())
                n_tot2 += n
        del sess, lg
    return n_cmp, n_tot, n_cmp2, n_tot2, bad


def test_hipmel_fixture_features_reproduce(gold):
    """The product's log-mel (kwhisper.WhisperFeatureExtractor on the GPU) of the fixture's stand-in clips, each
    zero-padded to 30 s, is BITWISE the features tests/golden/large_v3_c4_hipmel.npz holds (dumped on the GPU box by
    tools/dump_hipmel.py): the log-mel kernel's output is pinned, not only its tolerance to the oracle."""
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.synthetic import reazon_audio

    g = gold("large_v3_c4_hipmel")
    audio = np.zeros((len(g["clip_ids"]), 480000), np.float32)
    for j, (i, d) in enumerate(zip(g["clip_ids"], g["durations"])):
        c = reazon_audio(int(i), float(d))
        audio[j, : len(c)] = c
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins, device=torch.device("cuda", 0))
    got = fe.extract(torch.from_numpy(audio).cuda()).cpu().numpy()
    np.testing.assert_array_equal(got, g["features"])


def test_config4_hipmel_multipass(gold):
    """Config 4 on the PRODUCT's own inputs: tests/golden/large_v3_c4_hipmel.npz holds the HIP
    log-mel that kwhisper.WhisperFeatureExtractor gave stand-in clips 1 and 522 (three seek passes in the round-4
    engine's batch-32 scan, profiles/r04c_multipass_find.json) and six one-pass clips on the GPU box
    (tools/dump_hipmel.py), and transformers' fp32 / bf16 large-v3 run on exactly those features (tools/make_fixtures.py
    --only c4_hipmel; run_pseudo_labelling.py:99-102,268,338).  transformers takes ONE pass on every row of them, in
    fp32 and in bf16 (clip 522 decides one step by a margin of 0.0038).  The fp32 engine, through pseudo_label(), is
    bit-exact with transformers' fp32 tokens and per-row passes; the bf16 engine is teacher-forced along every fp32
    pass and its safe-margin greedy choice must equal the fp32 token (the engine's own passes, where they differ, are
    held to transformers' choices by test_config4_hipmel_engine_trajectory)."""
    g = gold("large_v3_c4_hipmel")
    feats = torch.from_numpy(g["features"]).cuda()
    n = feats.shape[0]
    m32 = _model(LARGE_V3, torch.float32)
    ids, preds = _c4_pseudo_label(m32, g["durations"], feats, n)
    assert ids == list(range(n))
    np.testing.assert_array_equal(np.stack(preds), g["tokens"])
    np.testing.assert_array_equal(m32.stats["row_passes"], g["passes"])
    print(f"\nconfig4 HIP log-mel fixture (clips {g['clip_ids'].tolist()}): transformers fp32 seek passes "
          f"{g['passes'].tolist()} (bf16 reference {g['bf16_passes'].tolist()}); fp32 engine bit-exact, same passes")
    del m32
    _free()
    m16 = _model(LARGE_V3, torch.bfloat16)
    n_cmp, n_tot, n_cmp2, n_tot2, bad = _teacher_forced_per_pass(m16, feats, g)
    t16 = m16.generate(feats, **C4_KW).cpu().numpy()
    print(f"config4 HIP log-mel bf16 teacher-forced per pass: {n_cmp} of {n_tot} steps compared (margin >= "
          f"{MARGIN_FLOOR}; passes >= 2: {n_cmp2} of {n_tot2}), {len(bad)} differ; free-running bf16 passes "
          f"{m16.stats['row_passes'].tolist()}, rows identical to fp32 "
          f"{sum(np.array_equal(a, b) for a, b in zip(t16, g['tokens']))}/{n}")
    assert len(bad) == 0, f"(pass entry, step) pairs whose safe-margin greedy choice differs: {bad[:8]}"
    assert n_cmp >= 0.9 * n_tot
    del m16
    _free()


def test_config4_seed6_short_clip_multipass(gold):
    """Config 4's seek advance INSIDE a zero-padded short clip at large-v3.  The fixture model
    (the numpy recipe's seed 0) takes one pass on all 1,768 stand-in clips, and so do seeds 1 (fp32 engine) and 2-5, 7-9
    (bf16 engine; profiles/r06d_*, r06e_multipass_scan_bf16.json); seed 6 takes two on 8 of the first batch's 32 clips, in the bf16 and in the fp32 engine (tools/find_multipass.py --seed
    6, profiles/r06f_multipass_fp32_seed6.json).  tests/golden/large_v3_c4_seed6.npz holds the HIP log-mel of 14 of
    them (8 multi-pass) from the GPU box and transformers' fp32 / bf16 large-v3 of seed 6 on exactly those features
    (tools/make_fixtures.py --only c4_seed --seed 6; run_pseudo_labelling.py:99-102,268,338): transformers takes two
    seek passes on the same 8 rows -- the mel re-encoded from the last complete segment's timestamp, the cumulative
    max_length growth (generation_whisper.py:785-903,1932-1940).  The fp32 engine through pseudo_label() is bit-exact
    with transformers' fp32 tokens AND per-row passes; the bf16 engine is teacher-forced along every fp32 pass, its
    safe-margin greedy choice equal to fp32's, passes >= 2 included."""
    g = gold("large_v3_c4_seed6")
    assert int(g["seed"]) == 6 and int((g["passes"] >= 2).sum()) >= 8
    feats = torch.from_numpy(g["features"]).cuda()
    n = feats.shape[0]
    m32 = _model(LARGE_V3, torch.float32, seed=6)
    ids, preds = _c4_pseudo_label(m32, g["durations"], feats, n)
    assert ids == list(range(n))
    np.testing.assert_array_equal(np.stack(preds), g["tokens"])
    np.testing.assert_array_equal(m32.stats["row_passes"], g["passes"])
    print(f"\nconfig4 seed-6 short clips {g['clip_ids'].tolist()}: transformers fp32 seek passes {g['passes'].tolist()} "
          f"(bf16 reference {g['bf16_passes'].tolist()}); fp32 engine bit-exact, same passes")
    del m32
    _free()
    m16 = _model(LARGE_V3, torch.bfloat16, seed=6)
    n_cmp, n_tot, n_cmp2, n_tot2, bad = _teacher_forced_per_pass(m16, feats, g)
    t16 = m16.generate(feats, **C4_KW).cpu().numpy()
    print(f"config4 seed-6 bf16 teacher-forced per pass: {n_cmp} of {n_tot} steps compared (margin >= {MARGIN_FLOOR}; "
          f"passes >= 2: {n_cmp2} of {n_tot2}), {len(bad)} differ; free-running bf16 passes "
          f"{m16.stats['row_passes'].tolist()}, rows identical to fp32 "
          f"{sum(np.array_equal(a, b) for a, b in zip(t16, g['tokens']))}/{n}")
    assert len(bad) == 0, f"(pass entry, step) pairs whose safe-margin greedy choice differs: {bad[:8]}"
    assert n_cmp >= 0.9 * n_tot and n_cmp2 > 0
    del m16
    _free()


@pytest.mark.parametrize("tag,floor", [("bf16", MARGIN_FLOOR), ("fp32", 1e-3)])
def test_config4_hipmel_engine_trajectory(gold, tag, floor):
    """Config 4's multi-pass case on the product's own inputs, along the ENGINE's trajectory.
    transformers decodes the HIP log-mel fixture in one seek pass per row; the bf16 engine follows fp32's choices
    only where fp32's margin exceeds the bf16 noise and so takes its own passes (up to three: a re-encode of the mel
    shifted to its last timestamp, generation_whisper.py:785-903, the cumulative max_length :1935-1940).
    tests/golden/large_v3_c4_hipmel_traj.npz holds the engine's passes recorded on the GPU box
    (tools/dump_trajectory.py) and transformers' fp32 choice and margin at every step of them, teacher-forced
    (tools/make_fixtures.py --only c4_traj).  The engine must reproduce its recorded passes exactly (rows, seek,
    frames, ids: deterministic), and at every step where fp32 decides by at least ``floor`` its token must be fp32's
    choice -- in every pass, the re-encoded later ones included."""
    g, t = gold("large_v3_c4_hipmel"), gold("large_v3_c4_hipmel_traj")
    if f"{tag}_pass_seq" not in t:
        pytest.skip(f"no {tag} trajectory in the fixture")
    feats = torch.from_numpy(g["features"]).cuda()
    m = _model(LARGE_V3, torch.bfloat16 if tag == "bf16" else torch.float32)
    m.record_pass_ids = True
    toks = m.generate(feats, **C4_KW).cpu().numpy()
    st = m.stats
    np.testing.assert_array_equal(st["row_passes"], t[f"{tag}_passes"])
    np.testing.assert_array_equal(toks, t[f"{tag}_tokens"])
    rows = [r for rr, _, _ in st["pass_log"] for r in rr]
    seeks = [x for _, ss, _ in st["pass_log"] for x in ss]
    nfr = [x for _, _, nn in st["pass_log"] for x in nn]
    np.testing.assert_array_equal(rows, t[f"{tag}_pass_row"])
    np.testing.assert_array_equal(seeks, t[f"{tag}_pass_seek"])
    np.testing.assert_array_equal(nfr, t[f"{tag}_pass_nframes"])
    seqs = [x for ids in st["pass_ids"] for x in ids]
    P = 3
    n_cmp = n_tot = n_cmp2 = n_tot2 = 0
    bad = []
    for k, x in enumerate(seqs):
        want = t[f"{tag}_pass_seq"][k]
        np.testing.assert_array_equal(x, want[: len(x)])
        n = int(t[f"{tag}_pass_len"][k])
        safe = t[f"{tag}_hf_margin"][k, :n] >= floor
        diff = np.nonzero(safe & (x[P: P + n] != t[f"{tag}_hf_choice"][k, :n]))[0]
        bad += [(k, int(d)) for d in diff]
        n_cmp += int(safe.sum())
        n_tot += n
        if t[f"{tag}_pass_iter"][k] >= 1:
            n_cmp2 += int(safe.sum())
            n_tot2 += n
    print(f"\nconfig4 HIP log-mel, {tag} engine trajectory: passes per row {st['row_passes'].tolist()}; {n_cmp} of "
          f"{n_tot} steps with transformers-fp32 margin >= {floor} compared (passes >= 2: {n_cmp2} of {n_tot2}), "
          f"{len(bad)} differ from fp32's choice")
    assert not bad, f"(pass entry, step) pairs off transformers' fp32 choice: {bad[:8]}"
    del m
    _free()


@pytest.mark.parametrize("fixture", ["large_v3_longform_fp32", "large_v3_longform8_fp32"])
def test_large_v3_longform_multipass(gold, fixture):
    """The seek loop's second and later passes at large-v3.  No config-4 stand-in clip takes a
    second pass under transformers' fp32 large-v3 at max_length 128 (all 1,768 scanned on the oracle log-mel,
    profiles/r04d_multipass_scan.json), so the multi-pass path -- the re-encode of the mel shifted to the last
    timestamp, the cumulative max_length growth (generation_whisper.py:785-903,1935-1940), the batch shrinking as
    rows finish -- is pinned on > 30 s clips batched with the frame mask at the config-4 settings
    (tests/golden/large_v3_longform_fp32.npz: 2 clips; large_v3_longform8_fp32.npz: 8 clips of 33-88 s): the fp32
    engine bit-exact with per-row pass counts equal to transformers' (>= 2 each), the bf16 engine margin-gated."""
    from _util import longform_inputs

    g = gold(fixture)
    feats, mask, _ = longform_inputs(g["clips"], n_mels=LARGE_V3.num_mel_bins)
    feats, mask = torch.from_numpy(feats).cuda(), torch.from_numpy(mask).cuda()
    kw = dict(language="ja", task="transcribe", return_timestamps=True, max_length=int(g["max_length"]))
    assert (g["passes"] >= 2).all()
    m32 = _model(LARGE_V3, torch.float32)
    toks = m32.generate(feats, attention_mask=mask, **kw).cpu().numpy()
    np.testing.assert_array_equal(toks, g["tokens"])
    np.testing.assert_array_equal(m32.stats["row_passes"], g["passes"])
    del m32
    _free()
    m16 = _model(LARGE_V3, torch.bfloat16)
    t16 = m16.generate(feats, attention_mask=mask, **kw).cpu().numpy()
    w = min(t16.shape[1], g["tokens"].shape[1])
    n = _gated_equal(t16[:, :w], g["tokens"][:, :w], g["margin"][:, :w])
    print(f"\n{fixture}: passes per row {g['passes'].tolist()} (fp32 engine bit-exact, same passes); bf16 free-running "
          f"{n} of {g['tokens'].size} tokens compared (margin >= {MARGIN_FLOOR}, up to each row's first unsafe step), "
          f"all equal; bf16 passes {m16.stats['row_passes'].tolist()}")
    # every pass, teacher-forced (the free-running gate stops each row at its first low margin)
    n_cmp, n_tot, n_cmp2, n_tot2, bad = _teacher_forced_per_pass(m16, feats, g)
    print(f"{fixture}: bf16 teacher-forced per pass: {n_cmp} of {n_tot} steps compared (passes >= 2: {n_cmp2} of "
          f"{n_tot2}), {len(bad)} differ")
    assert len(bad) == 0, f"(pass entry, step) pairs whose safe-margin greedy choice differs: {bad[:8]}"
    assert n_cmp2 > 0 and n_cmp >= 0.9 * n_tot
    del m16
    _free()


def test_lanes_cold_capture_multipass(gold):
    """lanes that start COLD -- no warm-up batch, so every session allocation and hipGraph capture
    (prefill, one step, K steps, for every batch size the seek loop shrinks to) happens on the lane threads while the
    other lane is running -- return exactly the one-lane results.  Two model.lane() handles decode the two halves of
    the eight-clip multi-pass long-form batch (passes 2-3 per row, batch 4 -> 3 -> ... rows) at the same time from
    two host threads, each on its own stream; captures are serialised by decode.CAPTURE_LOCK."""
    import threading

    from _util import longform_inputs

    g = gold("large_v3_longform8_fp32")
    feats, mask, _ = longform_inputs(g["clips"], n_mels=LARGE_V3.num_mel_bins)
    feats, mask = torch.from_numpy(feats).cuda(), torch.from_numpy(mask).cuda()
    kw = dict(language="ja", task="transcribe", return_timestamps=True, max_length=int(g["max_length"]))
    m16 = _model(LARGE_V3, torch.bfloat16)
    halves = [slice(0, 4), slice(4, 8)]
    lanes = [m16.lane(), m16.lane()]  # before any generate: nothing captured anywhere yet
    got, errs = [None, None], []
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    start = threading.Barrier(2)

    def run(i):
        try:
            with torch.cuda.stream(streams[i]):
                start.wait()
                got[i] = lanes[i].generate(feats[halves[i]], attention_mask=mask[halves[i]], **kw).cpu().numpy()
        except BaseException as e:
            errs.append(e)

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    torch.cuda.synchronize()
    for i, h in enumerate(halves):  # the one-lane reference (the caller's own handle, captured afterwards)
        want = m16.generate(feats[h], attention_mask=mask[h], **kw).cpu().numpy()
        np.testing.assert_array_equal(got[i], want, err_msg=f"lane {i}")
    print(f"\ncold lanes: two lanes captured their graphs concurrently (passes "
          f"{[lanes[i].stats['row_passes'].tolist() for i in range(2)]}); outputs equal the one-lane runs")
    del m16, lanes
    _free()


# The loop's host logic over the tiny engine (fixture-pinned first batch, W = 2, resume)

N_ITEMS, BS = 10, 4
GEN_KW = dict(language="ja", task="transcribe", return_timestamps=True, max_length=64)


def _items():
    """Items 0-3 are the tiny fixture clips (so batch 0 is pinned to the HF tokens), the rest other clips."""
    return ["dummy:0", "dummy:1", "tone:0", "tone:1"] + [f"dummy:{10 + i}" for i in range(N_ITEMS - 4)]


def _item_features(idx):
    return torch.from_numpy(oracle_features(TINY, [_items()[i] for i in idx])).cuda()


def _pad_to(rows, width, pad):
    out = np.full((len(rows), width), pad, dtype=np.int64)
    for i, r in enumerate(rows):
        out[i, : len(r)] = r
    return out


def _pl_worker(rank, world, port, out_dir):
    import torch.distributed as dist

    from kwhisper.pseudo_label import pseudo_label

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        model = _model(TINY, torch.float32)
        pad = model.generation_config.eos_token_id  # the tokenizer's pad id (<|endoftext|>), run_pseudo_labelling.py:339
        ids, preds = pseudo_label(model, _item_features, N_ITEMS, batch_size=BS, gen_kwargs=GEN_KW,
                                  pad_token_id=pad, comm_device="cpu")
        w = max(len(p) for p in preds)
        np.savez(os.path.join(out_dir, f"r{rank}.npz"), ids=np.array(ids), preds=_pad_to(preds, w, pad))
    finally:
        dist.destroy_process_group()


def test_config4_pseudo_label_engine(gold, tiny32, tmp_path):
    """run_pseudo_labelling.py:333-344 over the HIP engine with timestamps: W = 1 equals per-batch generate()
    (batch 0 = the HF fixture's greedy_ts tokens); W = 2 (two processes on this GPU, gloo) gathers the same
    predictions in dataset order."""
    import torch.multiprocessing as mp

    from kwhisper.pseudo_label import pseudo_label

    g = gold("tiny_fp32")
    pad = tiny32.generation_config.eos_token_id
    ids1, preds1 = pseudo_label(tiny32, _item_features, N_ITEMS, batch_size=BS, gen_kwargs=GEN_KW, pad_token_id=pad)
    assert ids1 == list(range(N_ITEMS))
    for b0 in range(0, N_ITEMS, BS):
        idx = list(range(b0, min(N_ITEMS, b0 + BS)))
        want = tiny32.generate(_item_features(idx), **GEN_KW).cpu().numpy()
        got = np.stack([preds1[i] for i in idx])
        np.testing.assert_array_equal(got, want)
    fx = tiny32.generate(_item_features(range(4)), language="ja", task="transcribe", return_timestamps=True,
                         max_length=int(g["max_length"])).cpu().numpy()
    np.testing.assert_array_equal(fx, g["greedy_ts_tokens"])  # the loop's inputs are the pinned clips
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_pl_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    w = max(len(p) for p in preds1)
    for r in range(2):
        z = np.load(tmp_path / f"r{r}.npz")
        assert z["ids"].tolist() == list(range(N_ITEMS))
        width = max(w, z["preds"].shape[1])
        np.testing.assert_array_equal(_pad_to(list(z["preds"]), width, pad), _pad_to(preds1, width, pad))
    print(f"\nconfig4 pseudo_label: W=1 and W=2 (gloo, 2 processes on cuda:0) agree on {N_ITEMS} items")


def test_config4_pseudo_label_resume_engine(tiny32, tmp_path):
    """Resume by round over the HIP engine: a run checkpoints its gathered rounds; after the last round's file
    is lost the rerun decodes that round only and returns the uninterrupted run's predictions."""
    from kwhisper.pseudo_label import pseudo_label

    pad = tiny32.generation_config.eos_token_id
    ck = str(tmp_path / "ck")
    ids1, preds1 = pseudo_label(tiny32, _item_features, N_ITEMS, batch_size=BS, gen_kwargs=GEN_KW, pad_token_id=pad,
                                checkpoint_dir=ck)
    last = sorted(f for f in os.listdir(ck) if f.startswith("round_"))[-1]
    os.remove(os.path.join(ck, last))
    seen = []
    ids2, preds2 = pseudo_label(tiny32, lambda idx: (seen.append(list(idx)), _item_features(idx))[1], N_ITEMS,
                                batch_size=BS, gen_kwargs=GEN_KW, pad_token_id=pad, checkpoint_dir=ck)
    assert seen == [[8, 9, 0, 1]]  # only the lost (wrapped) round was decoded again
    assert ids2 == ids1 == list(range(N_ITEMS))
    for a, b in zip(preds1, preds2):
        np.testing.assert_array_equal(a, b)


def test_pseudo_label_lanes_engine(tiny32):
    """pseudo_label(gather="end", lanes=2 / 3) over the HIP engine: batches decode concurrently on model.lane()
    handles from host threads, each on its own stream (graph capture thread-local, stream-local syncs); the
    predictions equal the one-lane run's, and step_model() names the handle that decoded each step."""
    from kwhisper.pseudo_label import pseudo_label, step_model

    pad = tiny32.generation_config.eos_token_id
    ids1, preds1 = pseudo_label(tiny32, _item_features, N_ITEMS, batch_size=BS, gen_kwargs=GEN_KW, pad_token_id=pad,
                                gather="end")
    for lanes in (2, 3):
        handles = {}

        def on_step(si, total):
            handles[si] = step_model()

        ids2, preds2 = pseudo_label(tiny32, _item_features, N_ITEMS, batch_size=BS, gen_kwargs=GEN_KW,
                                    pad_token_id=pad, gather="end", lanes=lanes, on_step=on_step)
        assert ids2 == ids1
        for a, b in zip(preds1, preds2):
            np.testing.assert_array_equal(a, b)
        assert len({id(h) for h in handles.values()}) == min(lanes, len(handles))
