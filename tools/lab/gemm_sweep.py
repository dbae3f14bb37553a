"""GEMM K / tile-count sweep (development): separates per-K-tile cost from per-tile overhead."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


res = {}
dev = "cuda"
for M, N in [(256 * 256, 256), (256 * 128, 512), (48000, 1280), (48000, 5120)]:
    for K in [320, 640, 1280, 2560]:
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        plan = ops.GemmPlan(A, W, C, M, N, K)
        us = t(plan)
        tiles = ((M + 255) // 256) * (N // 256)
        res[f"{M}x{N}x{K}"] = {"us": round(us, 1), "TF": round(2 * M * N * K / us / 1e6), "tiles": tiles}
        Z = torch.zeros_like(A)
        Wz = torch.zeros_like(W)
        us0 = t(ops.GemmPlan(Z, Wz, C, M, N, K))
        res[f"{M}x{N}x{K}"]["us_zeros"] = round(us0, 1)
print(json.dumps(res))
