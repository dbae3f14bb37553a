#!/usr/bin/env python
"""Encoder GEMM microbenchmark (development tool): TFLOP/s of kw_gemm at large-v3 B=32 shapes.

    KW_GEMM_TILE=128 KWHISPER_LIB=<lab build, -DKW_LAB_OVERRIDES> python tools/gemm_bench.py   # 128x128 kernel
    python tools/gemm_bench.py                    # default (256x256 ping-pong where it applies)
"""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import torch  # noqa: E402

from kwhisper import _lib as L  # noqa: E402
from kwhisper import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, T, d, F, H = 32, 1500, 1280, 5120, 20
    M = B * T
    res = {"tile": os.environ.get("KW_GEMM_TILE", "default")}
    x = torch.randn(M, F, device=dev).bfloat16()
    for name, N, K, epi in [("qkv_headsplit", 3 * d, d, L.KW_EPI_HEADSPLIT), ("o_resid", d, d, L.KW_EPI_RESID),
                            ("o_store_bf16", d, d, L.KW_EPI_STORE), ("fc2_store_bf16", d, F, L.KW_EPI_STORE),
                            ("fc1_gelu", F, d, L.KW_EPI_STORE), ("fc2_resid", d, F, L.KW_EPI_RESID),
                            ("cross_kv_headsplit", 2 * 32 * d, d, L.KW_EPI_HEADSPLIT)]:
        W = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        bias = torch.zeros(N, device=dev)
        A = x[:, :K].contiguous()
        kw = dict(bias=bias, epilogue=epi)
        if epi == L.KW_EPI_RESID:
            C = torch.zeros(M, N, device=dev)
        else:
            C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if epi == L.KW_EPI_HEADSPLIT:
            kw.update(hs_seq=T, hs_heads=H, hs_head_dim=64)
        if name == "fc1_gelu":
            kw["gelu"] = True
        plan = ops.GemmPlan(A, W, C, M, N, K, **kw)
        reps = 3 if N > 10000 else 10
        plan()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            plan()
        e1.record()
        e1.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        res[name] = {"us": round(us, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}
        # hipBLASLt on the same shape (plain GEMM, bf16 out, no epilogue) for reference
        if N <= 10000:
            torch.matmul(A, W.t())
            e0.record()
            for _ in range(reps):
                torch.matmul(A, W.t())
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            res[name + "_hipblaslt"] = {"us": round(us, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1)}
        del W, C
    # encoder self-attention: ours vs torch SDPA (flash/CK on ROCm)
    qkv = torch.randn(3, B, H, T, 64, device=dev).bfloat16() * 0.5
    out = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
    flops = 4 * B * H * T * T * 64
    for name, fn in [("attn", lambda: ops.attention(qkv, B, H, T, 64, out)),
                     ("attn_sdpa", lambda: torch.nn.functional.scaled_dot_product_attention(qkv[0], qkv[1], qkv[2]))]:
        try:
            fn()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 10
            res[name] = {"us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 1)}
        except Exception as e:  # noqa: BLE001
            res[name] = str(e)[:100]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
