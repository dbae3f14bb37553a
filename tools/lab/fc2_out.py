"""Lab: one fc2-shaped decode linear (N 1280, K 5120, RESID, B = 32) on fixed inputs, saved for a bitwise A/B of
two builds / env settings:  python tools/lab/fc2_out.py OUT.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(3)
B, N, K = 32, 1280, 5120
x = torch.randn(B, K, device="cuda", generator=g).bfloat16()
W = ops.pack_weight((torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16())
bias = torch.randn(N, device="cuda", generator=g)
h = torch.randn(B, N, device="cuda", generator=g)
hb = torch.empty(B, N, device="cuda", dtype=torch.bfloat16)
ws = torch.zeros(1 << 22, device="cuda")
ops.DecLinearPlan(x, W, B, N, K, bias=bias, workspace=ws, resid=(h, hb, N, 0))()
torch.cuda.synchronize()
torch.save({"h": h.cpu(), "hb": hb.cpu()}, sys.argv[1])
