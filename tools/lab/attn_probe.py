#!/usr/bin/env python
"""Encoder attention microbenchmark for the product kernel (lab r05w): kw_attention with KW_ATTN_Q_LOG2 (attn_fwd_l2,
the bf16 engine's) at large-v3 B = 32 (20 heads, 1500 frames), q scaled as the QKV epilogue scales it (hd^-0.5 log2 e).
Prints us per launch and TFLOP/s (tools/gemm_bench.py's "attn" row times the natural-unit kernel instead)."""
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
    B, H, T, hd = 32, 20, 1500, 64
    torch.manual_seed(0)
    qkv = torch.randn(3, B, H, T, hd, device=dev)
    qkv[0] *= hd ** -0.5 * 1.4426950408889634
    qkv = qkv.bfloat16()
    out = torch.empty(B * T, H * hd, device=dev, dtype=torch.bfloat16)
    fn = lambda: ops.attention(qkv, B, H, T, hd, out, q_log2=True)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        fn()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(json.dumps({"attn_l2_us": round(us, 1), "TFLOPs": round(4 * B * H * T * T * hd / us / 1e6, 1),
                      "checksum": float(out.float().abs().sum())}))


if __name__ == "__main__":
    main()
