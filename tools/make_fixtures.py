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


# ---------------------------------------------------------------------------------------------------------------
# Round 2: the measured workloads themselves (BASELINE configs 3 and 5)

B32_CASES = [("dummy", s) for s in range(16)] + [("tone", s) for s in range(16)]


def large_b32_fixtures():
    """tests/golden/large_v3_b32_fp32.npz: BASELINE config 3 itself -- large-v3, 32 clips, greedy,
    ``max_length=128`` (128 new tokens), no timestamps (run_pseudo_labelling.py:338 with the bench's
    gen_kwargs).  Stores the plain token matrix, per-step top-2 margins of the processed scores and the
    top-8 raw logits at every step (teacher-forced reference for the bf16 engine)."""
    t0 = time.time()
    m = hf_model(LARGE_V3)
    feats = features(LARGE_V3.num_mel_bins, B32_CASES)
    out = {"cases": np.array([f"{k}:{s}" for k, s in B32_CASES]), "max_length": 128}
    with torch.no_grad():
        enc = torch.cat([m.model.encoder(feats[i: i + 8]).last_hidden_state for i in range(0, 32, 8)])
    out["enc_slice"] = enc[:, ::250, :].numpy().astype(np.float32)
    out["enc_stats"] = np.stack([enc.double().sum((1, 2)).numpy(), (enc.double() ** 2).sum((1, 2)).numpy()], 1)
    del enc
    print(f"  large_v3_b32: encoder ({time.time() - t0:.1f}s)")
    kw = dict(language="ja", task="transcribe", return_timestamps=False, max_length=128)
    m.generation_config, _ = hf_gen_config(LARGE_V3)
    res = run_generate(m, feats, return_dict_in_generate=True, output_scores=True, output_logits=True, **kw)
    logits = torch.stack(res.logits, 1)
    top = logits.topk(8, -1)
    out["greedy_logits_top_idx"] = top.indices.numpy().astype(np.int32)
    out["greedy_logits_top_val"] = top.values.numpy().astype(np.float32)
    del logits, top
    s2 = torch.stack(res.scores, 1).topk(2, -1).values
    out["greedy_margin"] = (s2[..., 0] - s2[..., 1]).numpy().astype(np.float32)
    out["greedy_sequences"] = res.sequences.numpy().astype(np.int64)
    del res, s2
    print(f"  large_v3_b32: dict generate ({time.time() - t0:.1f}s)")
    m.generation_config, _ = hf_gen_config(LARGE_V3)
    out["greedy_tokens"] = run_generate(m, feats, **kw).numpy().astype(np.int64)
    np.savez_compressed(os.path.join(GOLD, "large_v3_b32_fp32.npz"), **out)
    print(f"large_v3_b32 fixtures done in {time.time() - t0:.1f}s {out['greedy_tokens'].shape}")


def large_bf16_ref_fixtures(rows=tuple(range(32))):
    """tests/golden/large_v3_bf16ref.npz: the REFERENCE's own bf16 noise floor at config 3.  The reference
    runs its teacher in bfloat16 (run_pseudo_labelling.py:229,338); here the same HF model is cast to bf16 on
    CPU and run on the 32 config-3 clips (round 2: rows 0 and 16 only): its encoder output, its teacher-forced logits on the fp32
    reference's token sequence (one decoder pass, at the fp32 top-8 ids) and its own greedy tokens.  The
    bf16 engine's tolerances are stated relative to these (tests/test_gpu_workloads.py)."""
    t0 = time.time()
    g = np.load(os.path.join(GOLD, "large_v3_b32_fp32.npz"))
    cases = [B32_CASES[r] for r in rows]
    m = hf_model(LARGE_V3).to(torch.bfloat16)
    feats = features(LARGE_V3.num_mel_bins, cases).to(torch.bfloat16)
    out = {"rows": np.array(rows), "cases": np.array([f"{k}:{s}" for k, s in cases])}
    with torch.no_grad():
        enc = m.model.encoder(feats).last_hidden_state
        out["enc_slice"] = enc[:, ::250, :].float().numpy()
        print(f"  large_v3_bf16ref: encoder ({time.time() - t0:.1f}s)")
        seq = torch.from_numpy(g["greedy_sequences"][list(rows), :-1])
        lg = m(encoder_outputs=(enc,), decoder_input_ids=seq).logits.float()[:, 3:]  # predicts seq[:, 4:] + 1
        idx = torch.from_numpy(g["greedy_logits_top_idx"][list(rows)].astype(np.int64))
        out["tf_logits_at_fp32_top8"] = torch.gather(lg[:, : idx.shape[1]], -1, idx).numpy().astype(np.float32)
        print(f"  large_v3_bf16ref: teacher-forced logits ({time.time() - t0:.1f}s)")
    m.generation_config, _ = hf_gen_config(LARGE_V3)
    out["greedy_tokens"] = run_generate(m, feats, language="ja", task="transcribe", return_timestamps=False,
                                        max_length=128).numpy().astype(np.int64)
    np.savez_compressed(os.path.join(GOLD, "large_v3_bf16ref.npz"), **out)
    print(f"large_v3_bf16ref fixtures done in {time.time() - t0:.1f}s")


C4_ITEMS = 32


def config4_audio(n=C4_ITEMS):
    """The first ``n`` clips of the config-4 stand-in (kwhisper.synthetic.reazon_durations / reazon_audio)."""
    durs = S.reazon_durations()[:n]
    return durs, [S.reazon_audio(i, float(d)) for i, d in enumerate(durs)]


def _aligned_margins(segs, P):
    """Per output token of one row, the top-1 / top-2 margin of the processed scores of the step that produced
    it.  A row's output is the concatenation over its seek passes of each pass's leading segment tokens
    (generation_whisper.py:2000-2074 slices segments from the start of the pass's sequence); every segment of
    one pass shares that pass's ``result`` (its sequences incl. the prompt, and per-step scores)."""
    groups = []
    for s in segs:
        if groups and groups[-1][0] is s["result"]:
            groups[-1][1].append(s)
        else:
            groups.append((s["result"], [s]))
    margins, toks = [], []
    for res, ss in groups:
        n = sum(len(s["tokens"]) for s in ss)
        gen = res["sequences"][P:]
        sc = torch.stack(list(res["scores"]), 0).float()  # (steps, V)
        assert n <= sc.shape[0]
        assert torch.equal(sc[:n].argmax(-1), gen[:n]), "greedy step != argmax of its scores"
        top = sc[:n].topk(2, -1).values
        margins.append((top[:, 0] - top[:, 1]).numpy())
        toks.append(gen[:n].numpy())
    return (np.concatenate(margins) if margins else np.zeros(0, np.float32),
            np.concatenate(toks) if toks else np.zeros(0, np.int64), len(groups))


def large_config4_fixtures():
    """tests/golden/large_v3_ts_b32_fp32.npz: BASELINE config 4's decode at its own teacher --
    run_pseudo_labelling.py:333-344 with its defaults (return_timestamps True, :99-102; batch 32,
    script/distil_whisper_v2.0.sh:32; max_label_length 128; ja / transcribe): HF fp32 large-v3 over the first
    32 clips of the ReazonSpeech-tiny duration stand-in (0.62-21.8 s, zero-padded to 30 s by the feature
    extractor).  Stores the token matrix, the per-token top-2 margins of the processed scores (aligned to the
    output through the seek passes), the number of seek passes per row and the segments."""
    t0 = time.time()
    durs, audio = config4_audio()
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins)
    feats = torch.from_numpy(fe(audio, sampling_rate=16000, return_tensors="np")["input_features"])
    m = hf_model(LARGE_V3)
    m.generation_config, gc = hf_gen_config(LARGE_V3)
    kw = dict(language="ja", task="transcribe", return_timestamps=True, max_length=128)
    res = run_generate(m, feats, return_dict_in_generate=True, output_scores=True, **kw)
    print(f"  large_v3_ts_b32: generate ({time.time() - t0:.1f}s)")
    toks = res["sequences"].numpy().astype(np.int64)
    P = 3  # [sot, ja, transcribe] (timestamps: no notimestamps token, generation_whisper.py:1591-1603)
    margin = np.full(toks.shape, np.inf, np.float32)
    passes = np.zeros(len(audio), np.int64)
    for b, segs in enumerate(res["segments"]):
        mg, tk, passes[b] = _aligned_margins(segs, P)
        assert np.array_equal(tk, toks[b, : len(tk)]) and (toks[b, len(tk):] == gc.pad_token_id).all()
        margin[b, : len(mg)] = mg
    segs = [[(float(x["start"]), float(x["end"]), len(x["tokens"])) for x in row] for row in res["segments"]]
    out = {"durations": durs.astype(np.float64), "tokens": toks, "margin": margin, "passes": passes,
           "segments": np.array(json.dumps(segs)), "max_length": 128}
    np.savez_compressed(os.path.join(GOLD, "large_v3_ts_b32_fp32.npz"), **out)
    print(f"large_v3_ts_b32 fixtures done in {time.time() - t0:.1f}s {toks.shape}, passes {passes.tolist()}")


class PassRecorder:
    """Records every iteration of transformers' seek loop (generation_whisper.py:785-903) on one model: which rows
    ran (batch_idx_map), each row's ``seek`` and ``seek_num_frames`` as ``_get_input_segment`` (:1831-1850) received
    them, and the per-row generate output of the pass (``generate_with_fallback``'s seek_outputs: the sequence with
    its prompt and the processed per-step scores).  Instance attributes shadow the two methods for one run."""

    def __init__(self, m):
        self.m, self.iters = m, []
        seg, gwf = type(m)._get_input_segment, m.generate_with_fallback

        def get_input_segment(input_features, seek, seek_num_frames, num_segment_frames, cur_bsz, batch_idx_map):
            rows = [int(batch_idx_map[i]) for i in range(cur_bsz)]
            self.iters.append({"rows": rows, "seek": [int(seek[r]) for r in rows],
                               "nframes": [int(seek_num_frames[r]) for r in rows]})
            return seg(input_features, seek, seek_num_frames, num_segment_frames, cur_bsz, batch_idx_map)

        def generate_with_fallback(**kw):
            out = gwf(**kw)
            self.iters[-1]["outputs"] = out[1]
            return out

        m._get_input_segment, m.generate_with_fallback = get_input_segment, generate_with_fallback

    def close(self):
        del self.m._get_input_segment, self.m.generate_with_fallback

    def arrays(self, P: int) -> dict:
        """One entry per (seek iteration, active row): pass_iter, pass_row, pass_seek, pass_nframes, pass_len
        (generated steps incl. a final EOS), pass_seq (prompt + generated, -1 padded) and pass_margin (top-1 - top-2
        of the processed scores at each step, +inf padded)."""
        ent = []
        for it, rec in enumerate(self.iters):
            for i, r in enumerate(rec["rows"]):
                o = rec["outputs"][i]
                sc = torch.stack(list(o["scores"]), 0).float()
                seq = o["sequences"].reshape(-1)[: P + sc.shape[0]]
                assert torch.equal(sc.argmax(-1), seq[P:]), "greedy step != argmax of its scores"
                top = sc.topk(2, -1).values
                ent.append((it, r, rec["seek"][i], rec["nframes"][i], seq.numpy(), (top[:, 0] - top[:, 1]).numpy()))
        T = max(len(e[4]) for e in ent)
        seqs = np.full((len(ent), T), -1, np.int64)
        marg = np.full((len(ent), T - P), np.inf, np.float32)
        for k, e in enumerate(ent):
            seqs[k, : len(e[4])] = e[4]
            marg[k, : len(e[5])] = e[5]
        return {"pass_iter": np.array([e[0] for e in ent], np.int64), "pass_row": np.array([e[1] for e in ent], np.int64),
                "pass_seek": np.array([e[2] for e in ent], np.int64),
                "pass_nframes": np.array([e[3] for e in ent], np.int64),
                "pass_len": np.array([len(e[5]) for e in ent], np.int64), "pass_seq": seqs, "pass_margin": marg}


def _c4_outputs(res, n_rows, P, gc):
    toks = res["sequences"].numpy().astype(np.int64)
    margin = np.full(toks.shape, np.inf, np.float32)
    passes = np.zeros(n_rows, np.int64)
    for b, segs in enumerate(res["segments"]):
        mg, tk, passes[b] = _aligned_margins(segs, P)
        assert np.array_equal(tk, toks[b, : len(tk)]) and (toks[b, len(tk):] == gc.pad_token_id).all()
        margin[b, : len(mg)] = mg
    segs = [[(float(x["start"]), float(x["end"]), len(x["tokens"])) for x in row] for row in res["segments"]]
    return toks, margin, passes, segs


def large_config4_hipmel_fixtures(features_npz, bf16=True, seed=0, name="large_v3_c4_hipmel"):
    """tests/golden/large_v3_c4_hipmel.npz: config 4's multi-pass case on the PRODUCT's own inputs (VERDICT r4 item
    1).  ``features_npz`` is tools/dump_hipmel.py's output from the GPU box: the exact f32 log-mel that the HIP feature
    extractor gives stand-in clips 1 and 522 (three seek passes in the fp32 engine, profiles/r04c_multipass_find.json)
    and six single-pass clips.  transformers' fp32 large-v3 decodes exactly those features with the reference's
    settings (run_pseudo_labelling.py:99-102,268,338; max_length 128 with the cumulative growth
    generation_whisper.py:1935-1940): tokens, per-token margins, seek passes per row, segments, and every pass's
    sequence / seek / margins (PassRecorder).  With ``bf16`` the same HF model cast to bfloat16 (the reference's own
    teacher precision, :229,338) also decodes them: its tokens and passes.

    r06: ``seed`` selects another model of the numpy recipe -- seed 6 is the first whose
    fp32 engine decodes short (zero-padded) stand-in clips in two seek passes (tools/find_multipass.py --seed 6,
    profiles/r06f_multipass_fp32_seed6.json) -- written as tests/golden/<name>.npz."""
    t0 = time.time()
    z = np.load(features_npz)
    feats = torch.from_numpy(z["features"].astype(np.float32))
    m = hf_model(LARGE_V3, seed)
    m.generation_config, gc = hf_gen_config(LARGE_V3)
    kw = dict(language="ja", task="transcribe", return_timestamps=True, max_length=128)
    rec = PassRecorder(m)
    res = run_generate(m, feats, return_dict_in_generate=True, output_scores=True, **kw)
    rec.close()
    P = 3
    toks, margin, passes, segs = _c4_outputs(res, feats.shape[0], P, gc)
    print(f"  {name}: fp32 generate ({time.time() - t0:.1f}s), passes {passes.tolist()}")
    out = {"clip_ids": z["clip_ids"], "durations": z["durations"], "features": z["features"].astype(np.float32),
           "tokens": toks, "margin": margin, "passes": passes, "segments": np.array(json.dumps(segs)),
           "max_length": 128, **rec.arrays(P)}
    if bf16:
        m.generation_config, _ = hf_gen_config(LARGE_V3)
        m = m.to(torch.bfloat16)
        r16 = PassRecorder(m)
        t16 = run_generate(m, feats.to(torch.bfloat16), return_segments=True, **kw)
        r16.close()
        out["bf16_tokens"] = t16["sequences"].numpy().astype(np.int64)
        out["bf16_passes"] = np.bincount([r for it in r16.iters for r in it["rows"]], minlength=feats.shape[0])
        print(f"  {name}: bf16 generate ({time.time() - t0:.1f}s), passes {out['bf16_passes'].tolist()}")
    out["seed"] = np.int64(seed)
    np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), **out)
    print(f"{name} fixtures done in {time.time() - t0:.1f}s {toks.shape}")


def large_config4_traj_fixtures(traj_npz):
    """tests/golden/large_v3_c4_hipmel_traj.npz: transformers' fp32 large-v3 scoring the ENGINE's own seek passes on
    the config-4 HIP log-mel fixture.  transformers decodes those features in one pass per row, the
    bf16 engine in up to three (its greedy choice follows fp32's only where fp32's margin exceeds the bf16 noise).
    ``traj_npz`` (tools/dump_trajectory.py, GPU box) holds every engine pass: rows, seek, frame count, ids.  For each
    pass the segment input is rebuilt from the fixture's features exactly as generation_whisper.py:1831-1850 cuts it,
    encoded by transformers, and the pass's ids fed through its decoder (teacher forcing); the logits are processed
    as the reference's greedy step processes them (oracle.generate.process_logits: Suppress -> SuppressAtBegin ->
    WhisperTimeStamp, pinned to transformers by tests/test_oracle_golden.py) and reduced to fp32's choice and its
    top-1 / top-2 margin at every step of the engine's trajectory."""
    sys.path.insert(0, ROOT)
    from oracle.generate import process_logits

    t0 = time.time()
    g = np.load(os.path.join(GOLD, "large_v3_c4_hipmel.npz"))
    tr = np.load(traj_npz)
    feats = torch.from_numpy(g["features"].astype(np.float32))
    m = hf_model(LARGE_V3)
    gd = generation_constants(LARGE_V3).to_dict()
    eos, P = gd["eos_token_id"], 3
    out = {}
    for tag in ("bf16", "fp32"):
        if f"{tag}_pass_seq" not in tr.files:
            continue
        seq_all = tr[f"{tag}_pass_seq"]
        n_ent, T = seq_all.shape
        choice = np.full((n_ent, T - P), -1, np.int64)
        margin = np.full((n_ent, T - P), np.inf, np.float32)
        length = np.zeros(n_ent, np.int64)
        for it in np.unique(tr[f"{tag}_pass_iter"]):
            ks = np.nonzero(tr[f"{tag}_pass_iter"] == it)[0]
            seg = torch.zeros((len(ks), feats.shape[1], 3000))
            for i, k in enumerate(ks):
                r, s0, nf = int(tr[f"{tag}_pass_row"][k]), int(tr[f"{tag}_pass_seek"][k]), int(tr[f"{tag}_pass_nframes"][k])
                seg[i, :, :nf] = feats[r, :, s0: s0 + nf]
            seq = seq_all[ks].copy()
            for i, k in enumerate(ks):  # generated steps: up to and including the first EOS
                body = seq[i, P:]
                valid = body[body >= 0]
                e = np.nonzero(valid == eos)[0]
                length[k] = int(e[0]) + 1 if e.size else len(valid)
            seq[seq < 0] = eos
            L = int(P + length[ks].max())
            with torch.no_grad():
                enc = m.model.encoder(seg).last_hidden_state
                lg = m(encoder_outputs=(enc,), decoder_input_ids=torch.from_numpy(seq[:, : L - 1])).logits.float().numpy()
            for i, k in enumerate(ks):
                for t in range(int(length[k])):
                    sc = process_logits(seq[i: i + 1, : P + t], lg[i, P - 1 + t][None], gd, P, True)[0]
                    top2 = np.partition(sc, -2)[-2:]
                    choice[k, t] = int(sc.argmax())
                    margin[k, t] = float(top2.max() - top2.min())
            print(f"  c4_traj {tag}: pass {it} ({len(ks)} rows) scored ({time.time() - t0:.1f}s)", flush=True)
        out.update({f"{tag}_{k}": tr[f"{tag}_{k}"] for k in ("tokens", "passes", "pass_iter", "pass_row", "pass_seek",
                                                             "pass_nframes", "pass_seq")})
        out.update({f"{tag}_pass_len": length, f"{tag}_hf_choice": choice, f"{tag}_hf_margin": margin})
    np.savez_compressed(os.path.join(GOLD, "large_v3_c4_hipmel_traj.npz"), **out)
    print(f"large_v3_c4_hipmel_traj fixtures done in {time.time() - t0:.1f}s")


LARGE_LONG_CLIPS = [("tone", 0, 45.0), ("dummy", 3, 70.0)]
# r04: eight more > 30 s clips (33-88 s) in one batch -- the multi-pass path on >= 8 rows
LARGE_LONG8_CLIPS = [("tone", 1, 38.0), ("dummy", 4, 52.0), ("tone", 2, 61.0), ("dummy", 5, 33.0),
                     ("tone", 3, 88.0), ("dummy", 6, 44.0), ("tone", 4, 57.0), ("dummy", 7, 75.0)]


def large_longform_fixtures(name="large_v3_longform_fp32", clips=None):
    """tests/golden/large_v3_longform_fp32.npz: the seek loop's SECOND and later passes at large-v3 (VERDICT r3 item
    1).  No config-4 stand-in clip takes a second pass in transformers' fp32 large-v3 at max_length 128 (every one of
    the 1,768 clips is single-pass: profiles/r04d_multipass_scan.json), so the multi-pass path -- re-encoding the mel
    shifted to the last timestamp, the cumulative max_length growth (generation_whisper.py:785-903,1935-1940), the
    shrinking batch -- is pinned on > 30 s clips, where every row takes several passes: two clips batched with the
    frame attention mask (the run_pseudo_labelling timestamp settings: ja / transcribe, max_length 128), tokens,
    per-token margins through the passes, passes per row, segments."""
    t0 = time.time()
    m = hf_model(LARGE_V3)
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins)
    clips = LARGE_LONG_CLIPS if clips is None else clips
    audio = [long_audio(k, s, sec) for k, s, sec in clips]
    inp = fe(audio, sampling_rate=16000, return_tensors="pt", truncation=False, padding="longest",
             return_attention_mask=True)
    m.generation_config, gc = hf_gen_config(LARGE_V3)
    rec = PassRecorder(m)  # r05: every pass's sequence / seek / margins, for the bf16 per-pass teacher-forced check
    res = run_generate(m, inp["input_features"], attention_mask=inp["attention_mask"], return_timestamps=True,
                       language="ja", task="transcribe", max_length=128, return_dict_in_generate=True,
                       output_scores=True)
    rec.close()
    print(f"  large_v3_longform: generate ({time.time() - t0:.1f}s)")
    P = 3
    toks, margin, passes, segs = _c4_outputs(res, len(audio), P, gc)
    out = {"clips": np.array([f"{k}:{s}:{sec}" for k, s, sec in clips]), "tokens": toks, "margin": margin,
           "passes": passes, "segments": np.array(json.dumps(segs)), "max_length": 128, **rec.arrays(P)}
    np.savez_compressed(os.path.join(GOLD, f"{name}.npz"), **out)
    print(f"{name} fixtures done in {time.time() - t0:.1f}s {toks.shape}, passes {passes.tolist()}")


KOTOBA_BEAM_CASES = [("tone", 0), ("dummy", 0), ("tone", 2), ("dummy", 3)]
KOTOBA_BEAM_MODES = [
    ("beam5_ts", dict(language="ja", task="transcribe", return_timestamps=True, num_beams=5, max_length=48)),
    ("beam5", dict(language="ja", task="transcribe", return_timestamps=False, num_beams=5, max_length=48)),
]


def kotoba_beam_fixtures():
    """tests/golden/kotoba_v2_beam_fp32.npz: BASELINE config 5's decode mode on the kotoba-whisper-v2.0
    layout (32 encoder / 2 decoder layers, script/distil_whisper_v2.0.sh:130-134): beam 5 with and without
    timestamps through the real HF generate (fp32, CPU)."""
    t0 = time.time()
    m = hf_model(KOTOBA_V2)
    feats = features(KOTOBA_V2.num_mel_bins, KOTOBA_BEAM_CASES)
    out = {"cases": np.array([f"{k}:{s}" for k, s in KOTOBA_BEAM_CASES])}
    for name, kw in KOTOBA_BEAM_MODES:
        m.generation_config, _ = hf_gen_config(KOTOBA_V2)
        out[f"{name}_tokens"] = run_generate(m, feats, **kw).numpy().astype(np.int64)
        print(f"  kotoba_v2_beam:{name} {out[f'{name}_tokens'].shape} ({time.time() - t0:.1f}s)")
    np.savez_compressed(os.path.join(GOLD, "kotoba_v2_beam_fp32.npz"), **out)


class _RecordingGenerate:
    """Wraps ``model.generate`` to keep every window batch the pipeline hands it (tokens as returned)."""

    def __init__(self, m):
        self.m, self.orig, self.calls = m, m.generate, []

    def __call__(self, *a, **kw):
        res = self.orig(*a, **kw)
        seq = res if isinstance(res, torch.Tensor) else res["sequences"]
        self.calls.append(seq.numpy().astype(np.int64))
        return res


def _stub_tokenizer(gen):
    """A stand-in tokenizer for the real ``AutomaticSpeechRecognitionPipeline`` (no vocab files offline):
    ids decode to "[id]" strings; the special ids and ``_decode_asr`` are transformers' own
    (tests/test_pipeline.py StubTokenizer)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import transformers.models.whisper.tokenization_whisper as tw
    from test_pipeline import StubTokenizer

    class Tok(StubTokenizer):
        pad_token_id = gen.pad_token_id
        eos_token_id = gen.eos_token_id
        padding_side = "right"

        def _decode_asr(self, model_outputs, *, return_timestamps, return_language, time_precision):
            return tw._decode_asr(self, model_outputs, return_timestamps=return_timestamps,
                                  return_language=return_language, time_precision=time_precision)

    tk = Tok(gen)
    tk.all_special_ids = tk.all_special_ids + [gen.pad_token_id]
    return tk


def pipeline_audio(spec):
    """"kind:seed:seconds" -> the seeded 30 s clips of ``kind`` concatenated and cut (long_audio); kind "reazon":
    clip ``seed`` of the config-4/5 stand-in at ``seconds`` (kwhisper.synthetic.reazon_audio, what
    tools/bench_configs.py feeds config 5)."""
    kind, seed, sec = str(spec).split(":")
    if kind == "reazon":
        return S.reazon_audio(int(seed), float(sec))
    return long_audio(kind, int(seed), float(sec))


PIPE_CASES = {
    # tag: (shape, clips, chunk_length_s, batch_size, generate_kwargs, return_timestamps values)
    "tiny": (TINY, ["dummy:0:40", "dummy:0:7"], 15, 3, dict(language="ja", task="transcribe", max_length=40),
             (False, True)),
    # no chunk_length_s: > 30 s clips go through the long-form seek loop, one item each (batched, masks)
    # (batch_size 1: transformers 5.15 cannot collate long-form items of different lengths, base.py:118)
    "tiny_longform": (TINY, [f"{k}:{s}:{sec}" for k, s, sec in LONG_CLIPS], None, 1,
                      dict(language="ja", task="transcribe"), (True,)),
    # BASELINE config 5 (run_short_form_eval.py:110-117,184-191 with chunk_length 15): kotoba-v2.0, beam 5
    "kotoba_v2": (KOTOBA_V2, ["tone:1:40", "dummy:5:12"], 15, 4,
                  dict(language="ja", task="transcribe", num_beams=5, max_length=40), (True,)),
    # config 5 at its BASELINE batch: 22 of tools/bench_configs.py's 30 s clips -> 66 windows,
    # window batches of 64 + 2 (bs = 64: 320 beam rows), beam 5, timestamps, max_length 128 as bench_configs runs it
    "kotoba_v2_b64": (KOTOBA_V2, [f"reazon:{i}:30" for i in range(22)], 15, 64,
                      dict(language="ja", task="transcribe", num_beams=5, max_length=128), (True,)),
    # the same pipeline with the model in bfloat16, as run_short_form_eval.py runs it on a GPU (torch_dtype bf16,
    # :110-117): the REFERENCE's own bf16 beam choices, the noise floor the bf16 engine is held to
    "kotoba_v2_b64_bf16": (KOTOBA_V2, [f"reazon:{i}:30" for i in range(22)], 15, 64,
                           dict(language="ja", task="transcribe", num_beams=5, max_length=128), (True,), torch.bfloat16),
}


def pipeline_fixtures(tags=("tiny", "tiny_longform", "kotoba_v2")):
    """tests/golden/pipeline_<tag>_fp32.npz: the REAL transformers ``pipeline("automatic-speech-recognition",
    chunk_length_s=..., batch_size=...)`` (automatic_speech_recognition.py:61-84,432-447,483-598) over the
    seeded HF model, with a stub tokenizer.  Stores the pipeline's final text / chunks (JSON) and every
    window batch's generate output."""
    from transformers import pipeline as hf_pipeline

    for tag in tags:
        t0 = time.time()
        shape, clips, chunk_s, bs, gk, ts_modes = PIPE_CASES[tag][:6]
        m = hf_model(shape)
        if len(PIPE_CASES[tag]) > 6:
            m = m.to(PIPE_CASES[tag][6])  # the pipeline casts the features to the model's dtype (chunk_iter :73-74)
        m.generation_config, gen = hf_gen_config(shape)
        rec = _RecordingGenerate(m)
        m.generate = rec
        fe = WhisperFeatureExtractor(feature_size=shape.num_mel_bins)
        pipe = hf_pipeline("automatic-speech-recognition", model=m, tokenizer=_stub_tokenizer(gen),
                           feature_extractor=fe, chunk_length_s=chunk_s, batch_size=bs, device="cpu")
        out = {"clips": np.array(clips), "batch_size": bs, "chunk_length_s": chunk_s or 0,
               "generate_kwargs": np.array(json.dumps(gk))}
        audio = [pipeline_audio(c) for c in clips]
        for ts in ts_modes:
            rec.calls.clear()
            with torch.no_grad():
                res = pipe([{"array": a, "sampling_rate": 16000} for a in audio], generate_kwargs=dict(gk),
                           return_timestamps=ts)
            key = f"ts{int(ts)}"
            out[f"{key}_result"] = np.array(json.dumps(res))
            out[f"{key}_n_calls"] = len(rec.calls)
            for i, c in enumerate(rec.calls):
                out[f"{key}_call{i}"] = c
            if len(PIPE_CASES[tag]) > 6:
                out["dtype"] = str(PIPE_CASES[tag][6])
            print(f"  pipeline_{tag}:{key} {len(rec.calls)} window batches ({time.time() - t0:.1f}s)")
        suffix = "" if len(PIPE_CASES[tag]) > 6 else "_fp32"  # (the bf16 case's tag says its dtype)
        np.savez_compressed(os.path.join(GOLD, f"pipeline_{tag}{suffix}.npz"), **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-large", action="store_true")
    ap.add_argument("--only", default=None)
    ap.add_argument("--hipmel", default="gpurun_out/c4_hipmel_features.npz",
                    help="--only c4_hipmel: tools/dump_hipmel.py output (the box's HIP log-mel of the chosen clips)")
    ap.add_argument("--no-bf16", action="store_true", help="--only c4_hipmel: skip the bf16 reference run")
    ap.add_argument("--seed", type=int, default=6, help="--only c4_seed: the numpy recipe's seed of the model")
    ap.add_argument("--traj", default="gpurun_out/c4_traj.npz",
                    help="--only c4_traj: tools/dump_trajectory.py output (the engine's seek passes on the fixture)")
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
    if not a.skip_large and a.only in (None, "large_b32"):
        large_b32_fixtures()
    if not a.skip_large and a.only in (None, "large_bf16ref"):
        large_bf16_ref_fixtures()
    if not a.skip_large and a.only in (None, "large_c4"):
        large_config4_fixtures()
    if not a.skip_large and a.only == "large_longform":
        large_longform_fixtures()
    if not a.skip_large and a.only == "large_longform8":
        large_longform_fixtures("large_v3_longform8_fp32", LARGE_LONG8_CLIPS)
    if not a.skip_large and a.only == "c4_hipmel":
        large_config4_hipmel_fixtures(a.hipmel, bf16=not a.no_bf16)
    if not a.skip_large and a.only == "c4_seed":  # r06: tests/golden/large_v3_c4_seed<seed>.npz
        large_config4_hipmel_fixtures(a.hipmel, bf16=not a.no_bf16, seed=a.seed, name=f"large_v3_c4_seed{a.seed}")
    if not a.skip_large and a.only == "c4_traj":
        large_config4_traj_fixtures(a.traj)
    if not a.skip_large and a.only in (None, "kotoba_beam"):
        kotoba_beam_fixtures()
    if a.only in (None, "pipeline"):
        pipeline_fixtures(("tiny", "tiny_longform") if a.skip_large else ("tiny", "tiny_longform", "kotoba_v2"))
    if not a.skip_large and a.only in (None, "pipeline_b64"):
        pipeline_fixtures(("kotoba_v2_b64",))
    if not a.skip_large and a.only in (None, "pipeline_b64_bf16"):
        pipeline_fixtures(("kotoba_v2_b64_bf16",))
    if not a.skip_large and a.only in (None, "kotoba"):
        cases = [("tone", 1), ("dummy", 2)]
        modes = [{"name": "greedy", "kw": dict(base, return_timestamps=False), "scores": True}]
        model_fixtures(KOTOBA_V2, "kotoba_v2_fp32", cases, 32, modes)


if __name__ == "__main__":
    main()
