#!/usr/bin/env python
"""Lab (not product): where the wall time of one bench batch goes outside the GPU kernels (large-v3, B = 32,
128 tokens).  Phases of generate() are bracketed by HIP events on the launch stream plus host timestamps.

    python tools/lab/host_gap_lab.py
"""
from __future__ import annotations

import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
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
    eng = model.engine
    s = torch.cuda.current_stream()

    # phase hooks: wrap engine.encode / cross_kv and the session's generate with events
    marks = []

    def ev(name):
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        marks.append((name, e, time.perf_counter()))

    enc0, ckv0 = eng.encode, eng.cross_kv

    def encode(*a, **k):
        ev("encode>")
        r = enc0(*a, **k)
        ev("encode<")
        return r

    def cross_kv(*a, **k):
        ev("cross_kv>")
        r = ckv0(*a, **k)
        ev("cross_kv<")
        return r

    eng.encode, eng.cross_kv = encode, cross_kv
    from kwhisper import decode as dmod
    gen0 = dmod.DecodeSession.generate

    def gen(self, *a, **k):
        ev("decode>")
        r = gen0(self, *a, **k)
        ev("decode<")
        return r

    dmod.DecodeSession.generate = gen
    for _ in range(2):
        model.generate(fe.extract(audio), **gen_kw)
    torch.cuda.synchronize()
    out = []
    for _ in range(3):
        marks.clear()
        t0 = time.perf_counter()
        ev("batch>")
        feats = fe.extract(audio)
        ev("features<")
        model.generate(feats, **gen_kw)
        ev("batch<")
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        first = marks[0][1]
        rows = {}
        prev = None
        for name, e, ht in marks:
            rows[name] = {"gpu_ms": round(first.elapsed_time(e), 3), "host_ms": round((ht - t0) * 1e3, 3)}
            prev = e
        rows["wall_ms"] = round((t1 - t0) * 1e3, 3)
        out.append(rows)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
