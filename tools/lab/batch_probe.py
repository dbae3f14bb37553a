#!/usr/bin/env python
"""Lab probe (not product): are config-4 rows the same at batch 32 and batch 8?  (r05: on the 8-clip HIP log-mel
fixture both engines decode clips 1 and 522 in one seek pass; the round-4 config-4 run at batch 32 took three on
batches 0 and 16, and the r04c fp32 scan found those clips three-pass.)  Decodes stand-in clips 0..31 (batch 0) and
512..543 (batch 16) at B = 32 and the fixture's 8 clips at B = 8 with the HIP log-mel, and compares the common rows.

    python tools/lab/batch_probe.py --dtype bfloat16
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="bfloat16")
    a = ap.parse_args()
    from kwhisper.config import LARGE_V3, generation_constants
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.synthetic import reazon_audio, reazon_durations, synthetic_state_dict

    dev = torch.device("cuda", 0)
    m = KWhisperForConditionalGeneration.from_state_dict(LARGE_V3, synthetic_state_dict(LARGE_V3, 0),
                                                         dtype=getattr(torch, a.dtype),
                                                         generation_config=generation_constants(LARGE_V3))
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins, device=dev)
    durs = reazon_durations()
    kw = dict(language="ja", task="transcribe", return_timestamps=True, max_length=128)

    def run(ids):
        audio = np.zeros((len(ids), 480000), np.float32)
        for j, i in enumerate(ids):
            c = reazon_audio(i, float(durs[i]))
            audio[j, : len(c)] = c
        feats = fe.extract(torch.from_numpy(audio).to(dev))
        toks = m.generate(feats, **kw).cpu().numpy()
        return toks, m.stats["row_passes"].tolist(), feats

    out = {"dtype": a.dtype}
    big = {}
    for b0 in (0, 512):
        ids = list(range(b0, b0 + 32))
        toks, passes, feats = run(ids)
        big.update({i: (toks[j], passes[j], feats[j]) for j, i in enumerate(ids)})
        out[f"b32_{b0}_passes"] = passes
    small = [1, 522, 0, 2, 3, 4, 5, 6]
    toks8, passes8, feats8 = run(small)
    out["b8_passes"] = passes8
    cmp = {}
    for j, i in enumerate(small):
        t32, p32, f32 = big[i]
        w = min(len(t32), len(toks8[j]))
        diff = np.nonzero(t32[:w] != toks8[j][:w])[0]
        cmp[i] = {"passes_b32": p32, "passes_b8": passes8[j], "same_features": bool(torch.equal(f32, feats8[j])),
                  "first_token_diff": int(diff[0]) if diff.size else None, "len": [int(len(t32)), int(len(toks8[j]))]}
    out["rows"] = cmp
    # the 8 rows again inside a batch of 32 made of them repeated (same rows, batch 32)
    feats32 = torch.cat([feats8] * 4)
    t = m.generate(feats32, **kw).cpu().numpy()
    out["b8x4_passes"] = m.stats["row_passes"].tolist()
    out["b8x4_rows_equal_b8"] = [bool(np.array_equal(t[j][: toks8.shape[1]], toks8[j])) for j in range(8)]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
