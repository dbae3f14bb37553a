#!/usr/bin/env python
"""Driver for tools/lab/xa_lab.hip: streaming ceilings of the decode cross-attention's K/V bytes by kernel
structure, beside the production kernel (kw_cross_attn_step), large-v3 B = 32: 32 distinct layers of
K/V [32][20][1500][64] bf16 (7.86 GB, so the 256 MB Infinity Cache cannot serve repeats)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402

B, H, S, HD, NL = 32, 20, 1500, 64, 32
dev = torch.device("cuda")
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "lab", "libxa_lab.so"))
lib.xa_lab_run.restype = ctypes.c_int
lib.xa_lab_run.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                           ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
K = [torch.randn(B, H, S, HD, device=dev).bfloat16() for _ in range(NL)]
V = [torch.randn(B, H, S, HD, device=dev).bfloat16() for _ in range(NL)]
out = torch.zeros(1 << 20, device=dev, dtype=torch.int32)
BYTES = 2 * B * H * S * HD * 2
res = {}


def timed(name, fn, reps=5):
    st = torch.cuda.current_stream()
    fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        for li in range(NL):
            fn(li)
    e1.record(st)
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (reps * NL)
    res[name] = {"us": round(us, 2), "TBps": round(BYTES / us / 1e6, 3)}
    print(f"{name:40s} {us:7.2f} us  {BYTES / us / 1e6:6.3f} TB/s", flush=True)


def lab(variant, per, ns, nwg=0):
    def fn(li):
        rc = lib.xa_lab_run(variant, per, K[li].data_ptr(), V[li].data_ptr(), B * H, S, ns, nwg, out.data_ptr(),
                            ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, rc
    return fn


q = torch.randn(B, H * HD, device=dev).bfloat16()
o = torch.empty(B, H * HD, device=dev, dtype=torch.bfloat16)
ws = torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, HD, S) // 4 + 1, device=dev)
timed("pair streaming (row kernel loads only)", lab(4, 8, 6))
timed("production pair kernel cross_attn_step", lambda li: ops.cross_attn_step(q, B, 1, H, HD, K[li], V[li], S, o, ws))
for ns, per in ((6, 8),):
    timed(f"reg  ns={ns} per={per}", lab(0, per, ns))
    timed(f"dma  ns={ns} per={per}", lab(1, per, ns))
    timed(f"kdma ns={ns} per={per}", lab(2, per, ns))
ncu = torch.cuda.get_device_properties(0).multi_processor_count
if os.environ.get("XA_LAB_LOOP"):
    for ns, per in ((6, 8), (12, 4), (24, 2)):
        for occ in (2, 4, 8):
            timed(f"loop ns={ns} per={per} wg={occ}/CU", lab(3, per, ns, ncu * occ))

timed("production cross_attn_step (end)", lambda li: ops.cross_attn_step(q, B, 1, H, HD, K[li], V[li], S, o, ws))
print(json.dumps(res))
