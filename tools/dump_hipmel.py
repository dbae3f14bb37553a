#!/usr/bin/env python
"""Dump the product's HIP log-mel of chosen config-4 stand-in clips (GPU box), for a transformers fixture.

Config 4's measured run (tools/bench_configs.py --config 4) feeds ``kwhisper.WhisperFeatureExtractor.extract`` of
each clip zero-padded to 30 s into generate() (run_pseudo_labelling.py:268,338).  On those features the fp32 engine
decodes stand-in clips 1 and 522 in THREE seek passes (profiles/r04c_multipass_find.json), while on the oracle log-mel
(within 2e-5) every stand-in clip takes one.  This writes the exact f32 features the engine saw, so that
tools/make_fixtures.py --only c4_hipmel can run transformers on exactly those inputs.

    python tools/dump_hipmel.py --clips 1,522,0,2,3,4,5,6 --out gpurun_out/c4_hipmel_features.npz
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", default="1,522,0,2,3,4,5,6")
    ap.add_argument("--out", default="gpurun_out/c4_hipmel_features.npz")
    a = ap.parse_args()
    from kwhisper.config import LARGE_V3
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.synthetic import reazon_audio, reazon_durations

    ids = [int(x) for x in a.clips.split(",")]
    durs = reazon_durations()
    audio = np.zeros((len(ids), 480000), np.float32)
    for j, i in enumerate(ids):
        c = reazon_audio(i, float(durs[i]))
        audio[j, : len(c)] = c
    dev = torch.device("cuda", 0)
    fe = WhisperFeatureExtractor(feature_size=LARGE_V3.num_mel_bins, device=dev)
    feats = fe.extract(torch.from_numpy(audio).to(dev)).cpu().numpy()
    # batch invariance of the log-mel: each clip alone gives its row of the batch
    for j in range(len(ids)):
        one = fe.extract(torch.from_numpy(audio[j: j + 1]).to(dev)).cpu().numpy()
        assert np.array_equal(one[0], feats[j]), f"log-mel row {j} depends on its batch"
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, clip_ids=np.asarray(ids, np.int64), durations=durs[ids].astype(np.float64),
                        features=feats.astype(np.float32))
    print(f"wrote {a.out}: {feats.shape} features of clips {ids} ({os.path.getsize(a.out) / 1e6:.2f} MB)", flush=True)


if __name__ == "__main__":
    main()
