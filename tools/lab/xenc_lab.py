"""Lab: time kw_cross_attn_enc variants (KWHISPER_LIB=<variant .so>, ctypes backend), B=32 large-v3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]
import torch  # noqa: E402

from kwhisper import ops  # noqa: E402

ops.set_backend("ctypes")
B, S, D, H = int(os.environ.get("XB", 32)), 1500, 1280, 20
enc = torch.randn(B, S, D, device="cuda").bfloat16()
u = (torch.randn(B, H * D, device="cuda") * 0.08).bfloat16()
z = torch.empty(B, H * D, device="cuda", dtype=torch.bfloat16)
ws = torch.zeros((ops.cross_attn_enc_workspace_bytes(B, D) + 3) // 4, device="cuda")
for _ in range(3):
    ops.cross_attn_enc(enc, B, S, D, u, 1, H, z, ws)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = 64
e0.record()
for _ in range(n):
    ops.cross_attn_enc(enc, B, S, D, u, 1, H, z, ws)
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) * 1e3 / n
print(f"{os.path.basename(os.environ.get('KWHISPER_LIB', 'libkwhisper.so'))} B={B}: {us:.2f} us/launch, "
      f"{B * S * D * 2 / us / 1e3:.0f} GB/s of e")

if os.environ.get("XSTAMPS"):
    import ctypes

    from kwhisper import _lib

    lib = _lib.load()
    buf = (ctypes.c_ulonglong * 1024)()
    ops.cross_attn_enc(enc, B, S, D, u, 1, H, z, ws)
    torch.cuda.synchronize()
    assert lib.kw_lab_xenc_stamps(buf) == 0
    for w in range(2):
        st = [buf[w * 512 + i] for i in range(512)]
        t0 = st[0]
        rel = lambda i: st[i] - t0 if st[i] else -1  # noqa: E731
        print(f"wave {2 * w}: u-loaded {rel(1)}, loop-end {rel(2)}, published {rel(3)}, synced {rel(4)}, "
              f"item-barrier {rel(5)}, merged {rel(6)}")
        for t in range(13):
            base = 8 + 8 * t
            if st[base] == 0:
                break
            ph = [st[base + k] for k in range(6)]
            print(f"  t={t}: start {ph[0] - t0}  S+write {ph[1] - ph[0]}  B1 {ph[2] - ph[1]}  fin {ph[3] - ph[2]}  "
                  f"B2 {ph[4] - ph[3]}  Z {ph[5] - ph[4]}")
