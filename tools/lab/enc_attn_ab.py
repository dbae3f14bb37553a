"""A/B of the encoder attention variants at large-v3 B = 32 (20 heads x 1500 frames): natural-unit q vs
KW_ATTN_Q_LOG2 (log2-unit q, reference subtracted on the matrix cores), HIP events over 10 launches."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402

B, H, T, hd = 32, 20, 1500, 64
qkv = (torch.randn(3, B, H, T, hd, device="cuda") * 0.5)
qkv[0] *= 0.125 * 8
q2 = qkv.clone()
q2[0] *= 1.4426950408889634
qkv, q2 = qkv.bfloat16(), q2.bfloat16()
out = torch.empty(B, T, H * hd, device="cuda", dtype=torch.bfloat16)
flop = 4 * B * H * T * T * hd
best = {}
for name, x, l2 in [("natural", qkv, False), ("log2 q", q2, True)] * 6:
    ops.attention(x, B, H, T, hd, out, q_log2=l2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.attention(x, B, H, T, hd, out, q_log2=l2)
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 100
    print(f"{name:8s} {us:8.1f} us/launch  {flop / us / 1e6:7.1f} TFLOP/s", flush=True)
    best[name] = min(best.get(name, 1e9), us)
print({k: round(v, 1) for k, v in best.items()})
