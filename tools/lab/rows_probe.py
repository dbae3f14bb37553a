#!/usr/bin/env python
"""kw_dec_linear above 32 rows (the weight-stationary row-chunk kernel: beam rows, prefill positions) -- device time
per call of the large-v3 decoder shapes at M = 128 (prefill: 32 items x 4 prompt positions) and M = 320 (64 windows x
5 beams), weights cycled over 8 copies so each call streams its weights as a decode step does.  Prints one JSON line.

    python tools/lab/rows_probe.py            # KWHISPER_LIB / KWHISPER_TORCH_LIB select the library under test
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
    d, F, NW, REPS = 1280, 5120, 8, 40
    out = {}
    for M in (128, 320):
        x = (torch.randn(M, F, device=dev) * 0.5).bfloat16()
        h = torch.randn(M, d, device=dev)
        hb = h.bfloat16()
        for name, N, K, kind in [("qkv_ln", 3 * d, d, "ln"), ("xq_ln", d, d, "ln"), ("fc1_ln_gelu", F, d, "gelu"),
                                 ("o_resid", d, d, "resid")]:
            plans = []
            for _ in range(NW):
                W = ops.pack_weight((torch.randn(N, K, device=dev) / K ** 0.5).bfloat16())
                bias = torch.randn(N, device=dev) * 0.01
                kw = dict(bias=bias)
                if kind in ("ln", "gelu"):
                    kw["ln"] = (1e-5, torch.randn(N, device=dev))  # (any column sums: timing only)
                    kw["C"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                    kw["gelu"] = kind == "gelu"
                else:
                    kw["resid"] = (h, hb, d, 0)
                plans.append(ops.DecLinearPlan(x, W, M, N, K, ldx=F, **kw))
            for p in plans:
                p()
            torch.cuda.synchronize()
            # one graph of REPS x NW calls: device time, no host launch gaps
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                with torch.cuda.graph(g, stream=s):
                    for r in range(REPS):
                        for p in plans:
                            p()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            e1.synchronize()
            out[f"{name}_M{M}"] = round(e0.elapsed_time(e1) * 1e3 / (REPS * NW), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
