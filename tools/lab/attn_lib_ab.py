#!/usr/bin/env python
"""Lab (not product): attn_fwd_l2 (kw_attention, KW_ATTN_Q_LOG2) output hashes and time with the library KWHISPER_LIB
points at -- A/B two builds for bitwise equality and speed.  Shapes: large-v3 B = 32 (T = 1500), ragged / short T, and
inputs whose scores grow along the keys (the exponent reference moves: the rare path).
    python tools/lab/attn_lib_ab.py"""
from __future__ import annotations

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]

import torch  # noqa: E402

hd = 64


def make(B, H, T, ramp=0.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    qkv = torch.randn(3, B, H, T, hd, device="cuda", generator=g) * 0.5
    qkv[0] *= 0.125 * 8 * 1.4426950408889634
    if ramp:
        qkv[1] *= (1.0 + ramp * torch.arange(T, device="cuda", dtype=torch.float32) / T)[None, None, :, None]
    return qkv.bfloat16().contiguous()


def main():
    from kwhisper import ops
    res = {"lib": os.environ.get("KWHISPER_LIB", "in-tree"), "sha": {}}
    for (B, H, T, ramp) in [(32, 20, 1500, 0.0), (2, 4, 1000, 0.0), (1, 2, 64, 0.0), (1, 2, 50, 0.0), (1, 3, 200, 0.0),
                            (2, 4, 1500, 6.0), (1, 2, 130, 12.0), (1, 2, 1, 0.0), (3, 5, 448, 3.0)]:
        x = make(B, H, T, ramp)
        out = torch.full((B, T, H * hd), float("nan"), device="cuda", dtype=torch.bfloat16)
        ops.attention(x, B, H, T, hd, out, q_log2=True)
        torch.cuda.synchronize()
        res["sha"][f"{B}x{H}x{T}r{ramp}"] = hashlib.sha256(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:12]
    B, H, T = 32, 20, 1500
    x = make(B, H, T)
    out = torch.empty(B, T, H * hd, device="cuda", dtype=torch.bfloat16)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(4):
        e0.record()
        for _ in range(10):
            ops.attention(x, B, H, T, hd, out, q_log2=True)
        e1.record()
        e1.synchronize()
        ts.append(round(e0.elapsed_time(e1) * 100, 1))
    res["us"] = ts
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
