"""r03au lab: does the decode step's cross-attention run faster when part of its layer's encoder K/V was read into
the Infinity Cache beforehand?  The cross block streams 245.8 MB per layer with non-temporal loads (no MALL
allocation) while the linears between two cross blocks leave HBM mostly idle (~42 us at ~0.8 TB/s); a
default-policy read of the next layer's K/V in that window would leave it MALL-resident.  Here, kernel level: one
layer's kw_dec_xq_cross timed (HIP events) after a cache flush, with 0 / 25 / 50 / 75 / 100 % of its K and V rows
(leading items) pre-read by a default-policy torch reduction."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402

dev = torch.device("cuda")
B, d, H, S = 32, 1280, 20, 1500
torch.manual_seed(0)
cross = torch.randn(2, B, H, S, 64, device=dev).bfloat16()
Wq = ops.pack_weight((torch.randn(d, d, device=dev) / d ** 0.5).bfloat16())
cs, bq = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
wsx = torch.zeros(ops.xq_cross_workspace_bytes(B, d, H, S) // 4 + 1, device=dev)
hb = torch.randn(B, d, device=dev).bfloat16()
out = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
plan = ops.XqCrossPlan(hb, Wq, B, d, H, ln=(1e-5, cs), bias=bq, scale=0.125, k=cross[0], v=cross[1], S=S, out=out,
                       workspace=wsx)
flush = torch.randn(600 * 1024 * 1024 // 2, device=dev).bfloat16()  # 600 MB, default-policy read evicts the MALL
sink = torch.zeros(4, device=dev)

plan()
torch.cuda.synchronize()
ref = out.clone()


def run(frac):
    sink[0] += flush.sum(dtype=torch.float32)
    rows = int(round(B * frac))
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    if rows:
        sink[1] += cross[0, :rows].sum(dtype=torch.float32)
        sink[2] += cross[1, :rows].sum(dtype=torch.float32)
    e1.record()
    plan()
    e2.record()
    e2.synchronize()
    return e0.elapsed_time(e1) * 1e3, e1.elapsed_time(e2) * 1e3


fracs = [0.0, 0.25, 0.5, 0.75, 1.0]
best = {f: 1e9 for f in fracs}
pre = {f: 0.0 for f in fracs}
for rnd in range(8):
    for f in fracs:
        tp, tc = run(f)
        if rnd:
            best[f] = min(best[f], tc)
            pre[f] = tp
print("output unchanged:", torch.equal(out, ref))
for f in fracs:
    print(f"pre-read {f:4.0%} of K/V rows: prefetch {pre[f]:7.1f} us, xq_cross {best[f]:6.2f} us (best of 7)", flush=True)

# residency check: the same default-policy read of 75 % of K (92 MB) right after a flush, then again
half = cross[0, :24]
for rnd in range(4):
    sink[0] += flush.sum(dtype=torch.float32)
    ts = []
    for _ in range(2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sink[3] += half.sum(dtype=torch.float32)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    print(f"92 MB default-policy read: cold {ts[0]:6.1f} us, repeated {ts[1]:6.1f} us", flush=True)
