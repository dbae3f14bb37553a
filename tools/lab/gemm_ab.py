#!/usr/bin/env python
"""Lab (not product): an encoder GEMM's output hash and time with the library KWHISPER_LIB points at (A/B two
builds for bitwise equality and speed).   python tools/lab/gemm_ab.py [fc1|qkv|o|fc2]"""
from __future__ import annotations

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]

import torch  # noqa: E402


def main():
    from kwhisper import _lib as L, ops
    which = sys.argv[1] if len(sys.argv) > 1 else "fc1"
    dev = torch.device("cuda")
    B, T, d, F, H = 32, 1500, 1280, 5120, 20
    M = B * T
    g = torch.Generator(device="cpu").manual_seed(1)
    N, K = {"fc1": (F, d), "qkv": (3 * d, d), "o": (d, d), "fc2": (d, F)}[which]
    A = (torch.randn((M, K), generator=g) * 1.0).to(torch.bfloat16).to(dev)
    W = (torch.randn((N, K), generator=g) / K ** 0.5).to(torch.bfloat16).to(dev)
    bias = (torch.randn((N,), generator=g) * 0.1).to(dev)
    C = torch.empty((M, N), device=dev, dtype=torch.bfloat16)
    kw = dict(bias=bias, gelu=which == "fc1")
    if which == "qkv":
        kw.update(epilogue=L.KW_EPI_HEADSPLIT, hs_seq=T, hs_heads=H, hs_head_dim=64, scale=0.125, scale_cols=d)
    plan = ops.GemmPlan(A, W, C, M, N, K, **kw)
    plan()
    torch.cuda.synchronize()
    h = hashlib.sha256(C.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        e0.record()
        for _ in range(10):
            plan()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 100)
    print(json.dumps({"gemm": which, "lib": os.environ.get("KWHISPER_LIB", "in-tree"), "sha": h,
                      "us": [round(t, 1) for t in ts]}), flush=True)


if __name__ == "__main__":
    main()
