#!/usr/bin/env python
"""Lab (not product): is the greedy decode step bound by the host's graph submission?  Large-v3, B = 32.
Captures the step graph through one generate(), then times N back-to-back replays on the GPU (events) and the
host's enqueue time for them (no sync inside the loop), with and without the per-step D2H flag copy.

    python tools/lab/replay_lab.py [--n 64]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    a = ap.parse_args()
    from kwhisper.config import PRESETS
    from kwhisper.feature_extraction import WhisperFeatureExtractor
    from kwhisper.generation import KWhisperForConditionalGeneration
    from kwhisper.synthetic import dummy_audio, synthetic_state_dict_torch

    dev = torch.device("cuda")
    shape = PRESETS["large-v3"]
    sd = synthetic_state_dict_torch(shape, seed=0, device=dev)
    model = KWhisperForConditionalGeneration.from_state_dict(shape, sd, dtype=torch.bfloat16, device=dev)
    del sd
    fe = WhisperFeatureExtractor(feature_size=shape.num_mel_bins, device=dev)
    audio = torch.from_numpy(np.stack([dummy_audio(i) for i in range(32)])).to(dev)
    gen_kw = dict(language="ja", task="transcribe", max_length=128, return_timestamps=False)
    model.generate(fe.extract(audio), **gen_kw)
    sess = next(iter(model._sessions.values()))
    g = sess._graph
    assert g is not None
    res = {}
    s = torch.cuda.current_stream()
    pinned = torch.zeros((8,), dtype=torch.int32).pin_memory()
    for mode in ("replay", "replay+flag", "replay", "replay+flag"):
        sess.cur_len.fill_(4)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        t0 = time.perf_counter()
        for i in range(a.n):
            g.replay()
            if mode == "replay+flag":
                pinned[i % 8: i % 8 + 1].copy_(sess.n_unfinished, non_blocking=True)
                torch.cuda.Event().record()
        t1 = time.perf_counter()
        e1.record(s)
        e1.synchronize()
        t2 = time.perf_counter()
        res.setdefault(mode, []).append({"gpu_ms_per_step": round(e0.elapsed_time(e1) / a.n, 4),
                                         "host_enqueue_ms_per_step": round((t1 - t0) * 1e3 / a.n, 4),
                                         "wall_ms_per_step": round((t2 - t0) * 1e3 / a.n, 4)})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
