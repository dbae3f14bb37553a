#!/usr/bin/env python
"""CPU fallback of tools/find_multipass.py: transformers 5.15.0 itself (fp32, CPU) decodes config-4 stand-in clips in
batches of 32 (return_timestamps=True, max_length 128, ja / transcribe -- run_pseudo_labelling.py:99-102,338) and
records each clip's number of seek passes (generation_whisper.py:785-903) until ``--need`` clips with >= 2 passes
are found.  Writes the same JSON layout as find_multipass.py ({"passes": [...]} for clips 0..n-1), which
tools/make_fixtures.py --only large_c4_mp consumes.  Build container only (imports transformers).

    PYTHONDONTWRITEBYTECODE=1 python tools/scan_multipass_cpu.py --start 32 --need 8 --out profiles/r04_multipass_clips.json
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
sys.path.insert(0, os.path.join(ROOT, "tools"))

import make_fixtures as mf  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--start", type=int, default=32, help="clips below this are known single-pass (r03 fixture)")
    ap.add_argument("--need", type=int, default=8)
    ap.add_argument("--max-clips", type=int, default=640)
    ap.add_argument("--out", default="profiles/r04_multipass_clips.json")
    a = ap.parse_args()
    torch.set_num_threads(os.cpu_count())
    durs = mf.S.reazon_durations()
    passes = [1] * a.start  # tests/golden/large_v3_ts_b32_fp32.npz: every one of the first 32 clips is single-pass
    m = mf.hf_model(mf.LARGE_V3)
    fe = mf.WhisperFeatureExtractor(feature_size=mf.LARGE_V3.num_mel_bins)
    t0 = time.time()
    for b0 in range(a.start, a.max_clips, 32):
        ids = list(range(b0, b0 + 32))
        audio = [mf.S.reazon_audio(i, float(durs[i])) for i in ids]
        feats = torch.from_numpy(fe(audio, sampling_rate=16000, return_tensors="np")["input_features"])
        m.generation_config, _ = mf.hf_gen_config(mf.LARGE_V3)
        res = mf.run_generate(m, feats, return_dict_in_generate=True, language="ja", task="transcribe",
                              return_timestamps=True, max_length=128)
        for segs in res["segments"]:
            groups = []
            for s in segs:
                if not groups or groups[-1] is not s["result"]:
                    groups.append(s["result"])
            passes.append(len(groups))
        n_multi = int((np.asarray(passes) >= 2).sum())
        print(f"clips {b0}-{b0 + 31}: passes {passes[-32:]} -> {n_multi} multi-pass so far ({time.time() - t0:.0f}s)",
              flush=True)
        with open(a.out, "w") as f:
            json.dump({"source": "transformers 5.15.0 fp32 CPU (tools/scan_multipass_cpu.py)", "n_clips": len(passes),
                       "max_length": 128, "passes": passes,
                       "multipass_clips": np.nonzero(np.asarray(passes) >= 2)[0].tolist()}, f)
        if n_multi >= a.need:
            break


if __name__ == "__main__":
    main()
