"""Pin the CPU oracle against golden vectors from the real reference path (transformers 5.15.0).

Fixtures: tests/golden/*.npz, produced by tools/make_fixtures.py.
"""
import numpy as np
import pytest

from kwhisper.config import KOTOBA_V2, LARGE_V3, TINY
from kwhisper.synthetic import synthetic_state_dict
from oracle import generate as og
from oracle.mel import log_mel, mel_filters
from oracle.whisper_np import WhisperNP

from _util import BEAM_MODES, TINY_MODES, audio_cases, beam_gen_dict, gen_dict, oracle_features, segments_of

STRIDE = 17


@pytest.mark.parametrize("n_mels", [80, 128])
def test_oracle_mel_filters(gold, n_mels):
    g = gold("mel_golden")
    np.testing.assert_allclose(mel_filters(n_mels), g[f"filters_{n_mels}"], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("n_mels", [80, 128])
def test_oracle_log_mel(gold, n_mels):
    g = gold("mel_golden")
    mel = log_mel(audio_cases(g["cases"]), n_mels)
    np.testing.assert_allclose(mel[:, :, ::STRIDE], g[f"mel_{n_mels}_slice"], atol=2e-5, rtol=0)
    stats = g[f"mel_{n_mels}_stats"]
    np.testing.assert_allclose(mel.sum((1, 2), dtype=np.float64), stats[:, 0], rtol=1e-6)
    np.testing.assert_allclose(mel.min((1, 2)), stats[:, 2], atol=2e-5)
    np.testing.assert_allclose(mel.max((1, 2)), stats[:, 3], atol=2e-5)


@pytest.mark.parametrize("n_mels", [80, 128])
def test_oracle_log_mel_edges(gold, n_mels):
    from oracle.mel import pad_or_trim
    from kwhisper import synthetic as S

    g = gold("mel_golden")
    edge = [S.tone_audio(2)[:24000], np.concatenate([S.tone_audio(3), S.dummy_audio(5)]), np.zeros(480000, np.float32)]
    mel = log_mel(np.stack([pad_or_trim(e) for e in edge]), n_mels)
    np.testing.assert_allclose(mel[:, :, ::STRIDE], g[f"edge_{n_mels}_slice"], atol=2e-5, rtol=0)
    np.testing.assert_allclose(mel[2], -1.5, atol=1e-6)  # silence: log10(1e-10) clamp -> (-10+4)/4


@pytest.fixture(scope="module")
def tiny():
    """The tiny oracle, its encoder memoised per mel (most tests here encode the same 4 clips; each numpy
    encode is seconds).  test_oracle_tiny_encoder, the first to ask, runs the real encoder."""
    m = WhisperNP(synthetic_state_dict(TINY, 0), TINY)
    encode, memo = m.encode, {}

    def cached(mel):
        mel = np.asarray(mel, dtype=np.float32)
        key = (mel.shape, hash(mel.tobytes()))
        if key not in memo:
            memo[key] = encode(mel)
        return memo[key].copy()

    m.encode = cached
    return m


def test_oracle_tiny_encoder(gold, tiny):
    g = gold("tiny_fp32")
    feats = oracle_features(TINY, g["cases"])
    enc = tiny.encode(feats)
    np.testing.assert_allclose(enc[:, ::50, :], g["enc_slice"], atol=2e-4, rtol=1e-4)


def test_oracle_tiny_logits(gold, tiny):
    """Teacher-forced on the fixture's token stream: per-step raw logits top-8 agree within 1e-3."""
    g = gold("tiny_fp32")
    feats = oracle_features(TINY, g["cases"])
    seq = g["greedy_sequences"]
    cache = tiny.new_cache(tiny.encode(feats))
    logits = tiny.decode(seq[:, :-1], cache)[:, 3:]  # positions predicting tokens 4..
    idx, val = g["greedy_logits_top_idx"], g["greedy_logits_top_val"]
    t = idx.shape[1]
    got = np.take_along_axis(logits[:, :t], idx.astype(np.int64), axis=-1)
    np.testing.assert_allclose(got, val, atol=1e-3, rtol=0)


@pytest.mark.parametrize("mode", sorted(TINY_MODES))
def test_oracle_tiny_generate(gold, tiny, mode):
    g = gold("tiny_fp32")
    kw, pad = TINY_MODES[mode]
    feats = oracle_features(TINY, g["cases"])
    kw = dict(kw)
    max_length = kw.pop("max_length", int(g["max_length"]))
    res = og.generate(tiny, feats, gen_dict(TINY, pad), max_length=max_length, **kw)
    toks = res["sequences"] if isinstance(res, dict) else res
    np.testing.assert_array_equal(toks, g[f"{mode}_tokens"])


@pytest.mark.parametrize("mode", sorted(BEAM_MODES))
def test_oracle_tiny_beam(gold, tiny, mode):
    """Beam search restatement vs HF generate (num_beams 2-5, EOS finishing, length penalty,
    early_stopping True / "never", timestamps)."""
    g = gold("tiny_beam_fp32")
    kw, eos = BEAM_MODES[mode]
    kw = dict(kw)
    feats = oracle_features(TINY, g["cases"])
    toks = og.generate(tiny, feats, beam_gen_dict(TINY, eos), max_length=kw.pop("max_length"), **kw)
    np.testing.assert_array_equal(toks, g[f"{mode}_tokens"])


def test_oracle_tiny_segments(gold, tiny):
    g = gold("tiny_fp32")
    feats = oracle_features(TINY, g["cases"])
    res = og.generate(tiny, feats, gen_dict(TINY), max_length=128, language="ja", task="transcribe",
                      return_timestamps=True, return_segments=True)
    want = segments_of(g["greedy_ts_segments_segments"])
    got = [[(s["start"], s["end"], len(s["tokens"])) for s in row] for row in res["segments"]]
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert [x[2] for x in a] == [x[2] for x in b]
        np.testing.assert_allclose([x[:2] for x in a], [x[:2] for x in b], atol=1e-9)


@pytest.mark.slow
@pytest.mark.parametrize("shape,tag", [(LARGE_V3, "large_v3_fp32"), (KOTOBA_V2, "kotoba_v2_fp32")])
def test_oracle_large_generate(gold, shape, tag):
    g = gold(tag)
    model = WhisperNP(synthetic_state_dict(shape, 0), shape)
    feats = oracle_features(shape, g["cases"])
    enc = model.encode(feats)
    np.testing.assert_allclose(enc[:, ::50, :], g["enc_slice"], atol=5e-4, rtol=1e-3)
    # generate re-encodes the same mel: serve it from the pass above (the numpy large encoder is minutes)
    encode, key = model.encode, feats.tobytes()
    model.encode = lambda x: enc if x.tobytes() == key else encode(x)
    toks = og.generate(model, feats, gen_dict(shape), max_length=int(g["max_length"]), language="ja",
                       task="transcribe", return_timestamps=False)
    np.testing.assert_array_equal(toks, g["greedy_tokens"])


@pytest.mark.slow
def test_oracle_tiny_longform(gold, tiny):
    """Long-form (> 3000 frames) seek loop: batched with an attention mask, and one clip without."""
    from _util import longform_inputs

    g = gold("tiny_longform_fp32")
    feats, mask, one = longform_inputs(g["clips"])
    res = og.generate(tiny, feats, gen_dict(TINY), language="ja", task="transcribe", return_timestamps=True,
                      attention_mask=mask, return_segments=True)
    np.testing.assert_array_equal(res["sequences"], g["long_ts_segments_tokens"])
    want = segments_of(g["long_ts_segments_segments"])
    got = [[(s["start"], s["end"], len(s["tokens"])) for s in row] for row in res["segments"]]
    assert [[x[2] for x in r] for r in got] == [[x[2] for x in r] for r in want]
    for rg, rw in zip(got, want):
        np.testing.assert_allclose([x[:2] for x in rg], [x[:2] for x in rw], atol=1e-9)
    np.testing.assert_array_equal(og.generate(tiny, one, gen_dict(TINY), language="ja", task="transcribe",
                                              return_timestamps=True), g["long_single_tokens"])
