#!/usr/bin/env python
"""Lab probe (not product): does a cross-attention launch run faster when its layer's K/V was just read
(Infinity Cache / MALL warm)?  Decides whether prefetching the next layer's cross K/V during the
dependent decode chain can pay.  Large-v3 shapes, B=32, S=1500.

    python tools/lab/mall_probe.py
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import torch  # noqa: E402

from kwhisper import ops  # noqa: E402


def graph_us(fns, reps=10):
    for f in fns:
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        for f in fns:
            f()
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    dev = torch.device("cuda")
    B, H, S, hd, nl = 32, 20, 1500, 64, 8
    d = H * hd
    cross = [torch.randn(2, B, H, S, hd, device=dev).bfloat16() for _ in range(nl)]
    q = torch.randn(B, d, device=dev).bfloat16()
    out = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
    ws = torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, hd, S) // 4 + 1, device=dev)
    red = torch.empty(nl, 4096, device=dev)

    def xa(i):
        return lambda: ops.cross_attn_step(q, B, 1, H, hd, cross[i][0], cross[i][1], S, out, ws)

    def touch(i, frac=1.0):
        flat = cross[i].view(-1)
        n = int(flat.numel() * frac) // 4096 * 4096
        return lambda: torch.sum(flat[:n].view(4096, -1), dim=1, dtype=torch.float32, out=red[i])

    res = {}
    res["cold_cross_us"] = graph_us([xa(i) for i in range(nl)]) / nl
    res["cross_twice_same_layer_us"] = graph_us([f for i in range(nl) for f in (xa(i), xa(i))]) / nl
    res["warm_cross_us (twice - cold)"] = res["cross_twice_same_layer_us"] - res["cold_cross_us"]
    for frac in (1.0, 0.5):
        t = graph_us([touch(i, frac) for i in range(nl)]) / nl
        tx = graph_us([f for i in range(nl) for f in (touch(i, frac), xa(i))]) / nl
        res[f"touch{frac}_us"] = t
        res[f"touch{frac}+cross_us"] = tx
        res[f"cross_after_touch{frac}_us"] = tx - t
    # prefetch of layer i+1 on a side stream while layer i's cross runs is not modelled here
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
