#!/usr/bin/env python
"""The all-rows LM head (lm_head_rows_kernel: beam rows, 33..320) -- device time per call vs the row count at large-v3
(N = 51866, K = 1280, LayerNorm folded, f32 logits), one weight copy (the weights stream from HBM each call: 133 MB
does not stay in the 256 MB Infinity Cache across the graph's other copies of nothing else).  One JSON line.
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import torch  # noqa: E402

from kwhisper import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N, K, REPS = 51866, 1280, 20
    W = ops.pack_weight((torch.randn(N, K, device=dev) / K ** 0.5).bfloat16())
    cs = torch.randn(N, device=dev)
    out = {}
    rows = [int(a) for a in sys.argv[1:]] or [32, 33, 64, 128, 192, 256, 320]  # (row counts on the command line)
    for M in rows:
        x = (torch.randn(M, K, device=dev) * 0.5).bfloat16()
        C = torch.empty(M, N, device=dev)
        plan = ops.DecLinearPlan(x, W, M, N, K, ln=(1e-5, cs), C=C)
        plan()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(REPS):
                    plan()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        out[f"M{M}"] = round(e0.elapsed_time(e1) * 1e3 / REPS, 1)
        del g, C
    print(json.dumps(out))


if __name__ == "__main__":
    main()
