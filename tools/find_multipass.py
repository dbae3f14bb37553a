#!/usr/bin/env python
"""Which config-4 stand-in clips take more than one seek pass at ``max_length`` 128 (GPU, fp32 parity mode).

The fp32 engine is bit-exact with transformers' fp32 generate (tests/test_gpu_workloads.py), so the clips it
decodes in >= 2 passes of the timestamp seek loop (generation_whisper.py:785-903, the cumulative max_length growth
:1935-1940) are the ones transformers also re-encodes.  tools/make_fixtures.py --only large_c4 then builds the
config-4 fixture over a 32-clip batch that contains such clips.

    python tools/find_multipass.py --n-clips 1768 --weights numpy --out gpurun_out/multipass.json \
        --features-out gpurun_out/multipass_features.npz
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-clips", type=int, default=640)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--out", default="gpurun_out/multipass.json")
    ap.add_argument("--weights", choices=("numpy", "torch"), default="numpy",
                    help="numpy: kwhisper.synthetic.synthetic_state_dict, the weights every transformers fixture uses; "
                    "torch: synthetic_state_dict_torch (the device generator: a DIFFERENT random model, which "
                    "transformers on the CPU cannot reproduce -- round 4's scan used it)")
    ap.add_argument("--seed", type=int, default=0, help="the numpy recipe's seed (the fixture model is seed 0)")
    ap.add_argument("--stop-after", type=int, default=0, help="stop once this many multi-pass clips were found (0: scan all)")
    ap.add_argument("--first-clip", type=int, default=0, help="scan clips [first-clip, first-clip + n-clips)")
    ap.add_argument("--features-out", default="",
                    help="npz of the HIP log-mel of every multi-pass clip (+ up to 8 one-pass clips) for "
                    "tools/make_fixtures.py --only c4_hipmel")
    a = ap.parse_args()
    from kwhisper.config import LARGE_V3, generation_constants
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.synthetic import reazon_audio, reazon_durations, synthetic_state_dict, synthetic_state_dict_torch

    dev = torch.device("cuda", 0)
    sd = (synthetic_state_dict(LARGE_V3, a.seed) if a.weights == "numpy"
          else synthetic_state_dict_torch(LARGE_V3, seed=a.seed, device=dev))
    model = KWhisperForConditionalGeneration.from_state_dict(LARGE_V3, sd, dtype=getattr(torch, a.dtype), device=dev,
                                                             generation_config=generation_constants(LARGE_V3))
    del sd
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins, device=dev)
    durs = reazon_durations()[: a.first_clip + a.n_clips]
    passes, ntok, keep = [], [], {}
    t0 = time.time()
    for b0 in range(a.first_clip, len(durs), a.batch):
        idx = list(range(b0, min(b0 + a.batch, len(durs))))
        audio = np.zeros((len(idx), 480000), np.float32)
        for j, i in enumerate(idx):
            c = reazon_audio(i, float(durs[i]))
            audio[j, : len(c)] = c
        feats = fe.extract(torch.from_numpy(audio).to(dev))
        toks = model.generate(feats, language="ja", task="transcribe", return_timestamps=True, max_length=128)
        pad = model.generation_config.pad_token_id
        rp = model.stats["row_passes"].tolist()
        for j, i in enumerate(idx):
            if rp[j] >= 2 or (len(keep) < 8 and i < 8):
                keep[i] = feats[j].cpu().numpy()
        passes += rp
        ntok += (toks != pad).sum(1).cpu().tolist()
        print(f"batch {b0 // a.batch}: passes {model.stats['row_passes'].tolist()} ({time.time() - t0:.1f}s)",
              flush=True)
        if a.stop_after and sum(1 for x in passes if x >= 2) >= a.stop_after:
            break
    passes = np.array(passes)
    if a.features_out and keep:
        ids = sorted(keep)
        np.savez_compressed(a.features_out, clip_ids=np.asarray(ids, np.int64), durations=durs[ids].astype(np.float64),
                            features=np.stack([keep[i] for i in ids]).astype(np.float32))
    res = {"dtype": a.dtype, "weights": a.weights, "seed": a.seed, "first_clip": a.first_clip, "n_clips": len(passes),
           "max_length": 128, "passes": passes.tolist(), "tokens": ntok,
           "multipass_clips": (a.first_clip + np.nonzero(passes >= 2)[0]).tolist(),
           "histogram": {int(k): int((passes == k).sum()) for k in np.unique(passes)}}
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f)
    print(json.dumps({k: res[k] for k in ("dtype", "weights", "n_clips", "histogram", "multipass_clips")}), flush=True)


if __name__ == "__main__":
    main()
