#!/usr/bin/env python
"""Lab (not product): where the prefill (4-token prompt, B = 32 rows x 4 positions, large-v3) goes -- the captured
prefill graph's replay time, and per-kernel device times of its launch sequence run eagerly with HIP events.

    python tools/lab/prefill_lab.py
"""
from __future__ import annotations

import json
import os
import sys

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
    model.generate(fe.extract(audio), **gen_kw)
    sess = next(iter(model._sessions.values()))
    cfg = next(iter(sess._greedy_cfg.values()))
    pg = cfg["prefill_graph"]
    P = 4
    s = torch.cuda.current_stream()
    res = {}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pg.replay()
    e0.record(s)
    for _ in range(10):
        pg.replay()
    e1.record(s)
    e1.synchronize()
    res["prefill_graph_ms"] = round(e0.elapsed_time(e1) / 10, 3)
    g = cfg["graph"]
    e0.record(s)
    for _ in range(10):
        g.replay()
    e1.record(s)
    e1.synchronize()
    res["step_graph_ms"] = round(e0.elapsed_time(e1) / 10, 3)
    seq = sess._step_plans(P)
    tot, cnt = {}, {}
    for _ in range(3):
        evs = []
        for item in seq:
            tag = item[0] if isinstance(item, tuple) else getattr(item, "tag", None) or "linear"
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            sess._run([item])
            b.record(s)
            evs.append((tag, a, b))
        evs[-1][2].synchronize()
        for tag, a, b in evs:
            tot[tag] = tot.get(tag, 0.0) + a.elapsed_time(b) * 1e3
            cnt[tag] = cnt.get(tag, 0) + 1
    res["prefill_kernel_us_avg"] = {k: round(tot[k] / cnt[k], 1) for k in tot}
    res["prefill_kernel_ms_total"] = {k: round(tot[k] / 3 / 1e3, 3) for k in tot}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
