#!/usr/bin/env python
"""Generate the golden vectors in tests/golden/ from the REAL reference code path.

The reference's hot path is transformers 5.15.0 (``WhisperFeatureExtractor``,
``WhisperForConditionalGeneration.generate``), imported here on CPU in fp32 with
the seeded synthetic weights of ``kwhisper.synthetic`` (no checkpoints exist
offline).  Run from the repo root in the build container:

    PYTHONDONTWRITEBYTECODE=1 python tools/make_fixtures.py [--skip-large]

Outputs are small .npz files: inputs are regenerable from seeds, so only
expected outputs (token matrices, logit top-k / margins, tensor slices and
full-tensor statistics) are stored.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

from kwhisper.config import KOTOBA_V2, LARGE_V3, TINY, generation_constants  # noqa: E402
from kwhisper import synthetic as S  # noqa: E402

from transformers import (  # noqa: E402
    GenerationConfig,
    WhisperConfig,
    WhisperFeatureExtractor,
    WhisperForConditionalGeneration,
)
from transformers.utils import logging as hf_logging  # noqa: E402

hf_logging.set_verbosity_error()
GOLD = os.path.join(ROOT, "tests", "golden")
MEL_STRIDE = 17


def hf_model(shape, seed=0):
    cfg = WhisperConfig(
        vocab_size=shape.vocab_size, num_mel_bins=shape.num_mel_bins, d_model=shape.d_model,
        encoder_layers=shape.encoder_layers, encoder_attention_heads=shape.encoder_attention_heads,
        encoder_ffn_dim=shape.encoder_ffn_dim, decoder_layers=shape.decoder_layers,
        decoder_attention_heads=shape.decoder_attention_heads, decoder_ffn_dim=shape.decoder_ffn_dim,
        decoder_start_token_id=shape.decoder_start_token_id, pad_token_id=shape.pad_token_id,
        eos_token_id=shape.eos_token_id, bos_token_id=shape.bos_token_id,
    )
    cfg._attn_implementation = "sdpa"
    m = WhisperForConditionalGeneration(cfg).eval()
    sd = {k: torch.from_numpy(v) for k, v in S.synthetic_state_dict(shape, seed).items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert missing == ["proj_out.weight"] and not unexpected, (missing, unexpected)
    return m


def hf_gen_config(shape, pad=None):
    gc = generation_constants(shape, pad_token_id=pad)
    d = {k: v for k, v in gc.to_dict().items() if k not in ("language", "task")}
    return GenerationConfig(**d), gc


def clip_audio(kind, seed):
    return getattr(S, f"{kind}_audio")(seed)


def mel_fixtures():
    out = {}
    cases = [("dummy", s) for s in range(4)] + [("tone", s) for s in range(2)]
    for n_mels in (80, 128):
        fe = WhisperFeatureExtractor(feature_size=n_mels)
        out[f"filters_{n_mels}"] = fe.mel_filters.astype(np.float64)
        audio = [clip_audio(k, s) for k, s in cases]
        feats = fe(audio, sampling_rate=16000, return_tensors="np")["input_features"]
        out[f"mel_{n_mels}_slice"] = feats[:, :, ::MEL_STRIDE].astype(np.float32)
        out[f"mel_{n_mels}_stats"] = np.stack(
            [feats.sum((1, 2), dtype=np.float64), (feats.astype(np.float64) ** 2).sum((1, 2)),
             feats.min((1, 2)).astype(np.float64), feats.max((1, 2)).astype(np.float64)], 1)
        # edge cases: short (zero-padded), long (truncated), digital silence
        edge = [clip_audio("tone", 2)[:24000], np.concatenate([clip_audio("tone", 3), clip_audio("dummy", 5)]),
                np.zeros(480000, np.float32)]
        ef = fe(edge, sampling_rate=16000, return_tensors="np")["input_features"]
        out[f"edge_{n_mels}_slice"] = ef[:, :, ::MEL_STRIDE].astype(np.float32)
    out["cases"] = np.array([f"{k}:{s}" for k, s in cases])
    np.savez_compressed(os.path.join(GOLD, "mel_golden.npz"), **out)
    print("mel fixtures done")


def features(n_mels, cases):
    fe = WhisperFeatureExtractor(feature_size=n_mels)
    audio = [clip_audio(k, s) for k, s in cases]
    return torch.from_numpy(fe(audio, sampling_rate=16000, return_tensors="np")["input_features"])


def run_generate(m, feats, **kw):
    with torch.no_grad():
        return m.generate(feats, **kw)


def model_fixtures(shape, tag, cases, max_length, modes, enc_rows=50):
    t0 = time.time()
    m = hf_model(shape)
    feats = features(shape.num_mel_bins, cases)
    out = {"cases": np.array([f"{k}:{s}" for k, s in cases]), "max_length": max_length}
    with torch.no_grad():
        enc = m.model.encoder(feats).last_hidden_state
    out["enc_slice"] = enc[:, ::enc_rows, :].numpy().astype(np.float32)
    out["enc_stats"] = np.stack([enc.double().sum((1, 2)).numpy(), (enc.double() ** 2).sum((1, 2)).numpy()], 1)
    for mode in modes:
        name, kw, pad = mode["name"], dict(mode["kw"]), mode.get("pad")
        gconf, _ = hf_gen_config(shape, pad)
        m.generation_config = gconf
        kw.setdefault("max_length", max_length)
        if mode.get("scores"):
            res = run_generate(m, feats, return_dict_in_generate=True, output_scores=True, output_logits=True, **kw)
            seq = res["sequences"] if isinstance(res, dict) else res.sequences
            logits = torch.stack(res.logits, 1).float()  # (B, T, V) raw
            scores = torch.stack(res.scores, 1).float()
            top = logits.topk(8, -1)
            out[f"{name}_logits_top_idx"] = top.indices.numpy().astype(np.int32)
            out[f"{name}_logits_top_val"] = top.values.numpy().astype(np.float32)
            s2 = scores.topk(2, -1).values
            out[f"{name}_margin"] = (s2[..., 0] - s2[..., 1]).numpy().astype(np.float32)
            out[f"{name}_sequences"] = seq.numpy().astype(np.int64)
            # plain (non-dict) call for the default output layout
            m.generation_config, _ = hf_gen_config(shape, pad)
            out[f"{name}_tokens"] = run_generate(m, feats, **kw).numpy().astype(np.int64)
        else:
            res = run_generate(m, feats, **kw)
            if isinstance(res, torch.Tensor):
                out[f"{name}_tokens"] = res.numpy().astype(np.int64)
            else:
                out[f"{name}_tokens"] = res["sequences"].numpy().astype(np.int64)
                if "segments" in res:
                    segs = [[(float(s["start"]), float(s["end"]), len(s["tokens"])) for s in row] for row in res["segments"]]
                    out[f"{name}_segments"] = np.array(json.dumps(segs))
        print(f"  {tag}:{name} {out[f'{name}_tokens'].shape} ({time.time() - t0:.1f}s)")
    np.savez_compressed(os.path.join(GOLD, f"{tag}.npz"), **out)
    print(f"{tag} fixtures done in {time.time() - t0:.1f}s")


BEAM_MODES = [
    # name, generate kwargs, eos override (a token the random-init tiny model emits often, so beams finish)
    ("beam5_ts", dict(return_timestamps=True, num_beams=5, max_length=40), None),
    ("beam3_eos", dict(return_timestamps=False, num_beams=3, max_length=40), 7656),
    ("beam4_eos_lp_es", dict(return_timestamps=False, num_beams=4, max_length=40, length_penalty=0.5,
                             early_stopping=True), 7656),
    ("beam2_eos_never", dict(return_timestamps=False, num_beams=2, max_length=40, length_penalty=2.0,
                             early_stopping="never"), 20779),
    ("beam3_eos_ts", dict(return_timestamps=True, num_beams=3, max_length=40), 7656),
]


def beam_fixtures():
    """tests/golden/tiny_beam_fp32.npz: beam search through the real HF generate (tiny, fp32)."""
    t0 = time.time()
    m = hf_model(TINY)
    cases = [("dummy", 0), ("dummy", 1), ("tone", 0), ("tone", 1)]
    feats = features(TINY.num_mel_bins, cases)
    out = {"cases": np.array([f"{k}:{s}" for k, s in cases])}
    for name, kw, eos in BEAM_MODES:
        gconf, _ = hf_gen_config(TINY)
        if eos is not None:
            gconf.eos_token_id = eos
        m.generation_config = gconf
        res = run_generate(m, feats, language="ja", task="transcribe", **kw)
        out[f"{name}_tokens"] = res.numpy().astype(np.int64)
        print(f"  tiny_beam:{name} {tuple(res.shape)} ({time.time() - t0:.1f}s)")
    np.savez_compressed(os.path.join(GOLD, "tiny_beam_fp32.npz"), **out)


LONG_CLIPS = [("tone", 0, 45.0), ("dummy", 3, 70.0), ("dummy", 4, 12.0)]


def long_audio(kind, seed, seconds):
    """> 30 s clips for the long-form seek loop: the seeded 30 s clips of ``kind`` concatenated."""
    n = int(seconds * 16000)
    parts, k = [], 0
    while sum(len(p) for p in parts) < n:
        parts.append(clip_audio(kind, seed + 10 * k))
        k += 1
    return np.concatenate(parts)[:n].astype(np.float32)


def longform_fixtures():
    """tests/golden/tiny_longform_fp32.npz: long-form (> 3000 frames) generate through the real HF seek loop
    (generation_whisper.py:785-903): batched with an attention mask, and a single clip without one."""
    t0 = time.time()
    m = hf_model(TINY)
    fe = WhisperFeatureExtractor(feature_size=TINY.num_mel_bins)
    audio = [long_audio(k, s, sec) for k, s, sec in LONG_CLIPS]
    inp = fe(audio, sampling_rate=16000, return_tensors="pt", truncation=False, padding="longest",
             return_attention_mask=True)
    out = {"clips": np.array([f"{k}:{s}:{sec}" for k, s, sec in LONG_CLIPS])}
    for name, kw in [("long_ts", dict(language="ja", task="transcribe")),
                     ("long_ts_segments", dict(language="ja", task="transcribe", return_segments=True))]:
        m.generation_config, _ = hf_gen_config(TINY)
        res = run_generate(m, inp["input_features"], attention_mask=inp["attention_mask"], return_timestamps=True,
                           **kw)
        if isinstance(res, torch.Tensor):
            out[f"{name}_tokens"] = res.numpy().astype(np.int64)
        else:
            out[f"{name}_tokens"] = res["sequences"].numpy().astype(np.int64)
            segs = [[(float(x["start"]), float(x["end"]), len(x["tokens"])) for x in row] for row in res["segments"]]
            out[f"{name}_segments"] = np.array(json.dumps(segs))
        print(f"  tiny_longform:{name} {tuple(out[f'{name}_tokens'].shape)} ({time.time() - t0:.1f}s)")
    one = fe([audio[1]], sampling_rate=16000, return_tensors="pt", truncation=False, padding="longest")
    m.generation_config, _ = hf_gen_config(TINY)
    res = run_generate(m, one["input_features"], return_timestamps=True, language="ja", task="transcribe")
    out["long_single_tokens"] = res.numpy().astype(np.int64)
    np.savez_compressed(os.path.join(GOLD, "tiny_longform_fp32.npz"), **out)
    print(f"tiny_longform fixtures done in {time.time() - t0:.1f}s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-large", action="store_true")
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    os.makedirs(GOLD, exist_ok=True)
    torch.manual_seed(0)
    torch.set_num_threads(os.cpu_count())
    if a.only in (None, "mel"):
        mel_fixtures()
    base = dict(language="ja", task="transcribe")
    tiny_modes = [
        {"name": "greedy", "kw": dict(base, return_timestamps=False), "scores": True},
        {"name": "greedy_ts", "kw": dict(base, return_timestamps=True)},
        {"name": "greedy_ts_segments", "kw": dict(base, return_timestamps=True, return_segments=True)},
        {"name": "greedy_dict", "kw": dict(base, return_timestamps=False, return_dict_in_generate=True)},
        {"name": "greedy_pad_eq_eos", "kw": dict(base, return_timestamps=True), "pad": 50257},
        {"name": "greedy_translate", "kw": dict(language="ja", task="translate", return_timestamps=False)},
        {"name": "greedy_detect", "kw": dict(return_timestamps=False)},
        {"name": "greedy_short", "kw": dict(base, return_timestamps=False, max_length=16)},
        {"name": "beam5", "kw": dict(base, return_timestamps=False, num_beams=5, max_length=24)},
    ]
    if a.only in (None, "beam"):
        beam_fixtures()
    if a.only in (None, "longform"):
        longform_fixtures()
    if a.only in (None, "tiny"):
        cases = [("dummy", 0), ("dummy", 1), ("tone", 0), ("tone", 1)]
        model_fixtures(TINY, "tiny_fp32", cases, 128, tiny_modes)
    if not a.skip_large and a.only in (None, "large"):
        cases = [("tone", 0), ("dummy", 0)]
        modes = [{"name": "greedy", "kw": dict(base, return_timestamps=False), "scores": True},
                 {"name": "greedy_ts", "kw": dict(base, return_timestamps=True, max_length=24)}]
        model_fixtures(LARGE_V3, "large_v3_fp32", cases, 32, modes)
    if not a.skip_large and a.only in (None, "kotoba"):
        cases = [("tone", 1), ("dummy", 2)]
        modes = [{"name": "greedy", "kw": dict(base, return_timestamps=False), "scores": True}]
        model_fixtures(KOTOBA_V2, "kotoba_v2_fp32", cases, 32, modes)


if __name__ == "__main__":
    main()
