#!/usr/bin/env python
"""Lab (not product): kw_dec_linear outputs on fixed seeded inputs for every decode-step shape (o / xo, fc1, fc2 with its
K-split seam, qkv, xq, LM head) at several row counts, saved to an npz -- run once per library (KWHISPER_LIB /
KWHISPER_TORCH_LIB) and compare: a restructured epilogue or seam must give the same bits.

    python tools/lab/declin_bitwise.py out.npz            # dump
    python tools/lab/declin_bitwise.py --compare a.npz b.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import numpy as np  # noqa: E402


def dump(path):
    import torch

    from kwhisper import ops

    out = {}
    g = torch.Generator(device="cuda").manual_seed(1234)
    shapes = [("o", 1280, 1280, "resid"), ("fc1", 5120, 1280, "gelu"), ("fc2", 1280, 5120, "resid"),
              ("qkv", 3840, 1280, "ln"), ("lm", 51866, 1280, "lm")]
    for name, N, K, mode in shapes:
        W = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
        Wp = ops.pack_weight(W)
        cs = ops.ln_colsum(W)
        b = torch.randn(N, device="cuda", generator=g) * 0.1
        ws = torch.zeros(ops.dec_linear_workspace_bytes(N, K) // 4 + 1, device="cuda")
        for M in (1, 5, 16, 17, 32, 64, 70, 128, 320):
            x = (torch.randn(M, K, device="cuda", generator=g) * 2 + 0.3).bfloat16()
            if mode == "resid":
                h = torch.randn(M, N, device="cuda", generator=g)
                hb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                for _ in range(2):  # twice: the seam counters come back to zero
                    hh = h.clone()
                    ops.DecLinearPlan(x, Wp, M, N, K, bias=b, resid=(hh, hb, N, 0), workspace=ws)()
                out[f"{name}_{M}_h"] = hh.cpu().numpy()
                out[f"{name}_{M}_hb"] = hb.view(torch.int16).cpu().numpy()
            else:
                dt = torch.bfloat16 if mode == "gelu" else torch.float32
                C = torch.empty(M, N, device="cuda", dtype=dt)
                ops.DecLinearPlan(x, Wp, M, N, K, ln=(1e-5, cs), bias=b, C=C, gelu=mode == "gelu", workspace=ws,
                                  scale=0.125 if mode == "ln" else 1.0, scale_cols=1280 if mode == "ln" else 0)()
                out[f"{name}_{M}_C"] = (C.view(torch.int16) if dt == torch.bfloat16 else C).cpu().numpy()
    torch.cuda.synchronize()
    np.savez(path, **out)
    print(f"dumped {len(out)} arrays to {path}")


def compare(a, b):
    za, zb = np.load(a), np.load(b)
    bad = [k for k in za.files if not np.array_equal(za[k], zb[k], equal_nan=True)]
    print(f"{len(za.files)} arrays compared, {len(bad)} differ: {bad}")
    return not bad


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(0 if compare(sys.argv[2], sys.argv[3]) else 1)
    dump(sys.argv[1])
