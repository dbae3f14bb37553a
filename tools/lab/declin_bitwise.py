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
    # decode attention (r06: the cross / self helpers' reductions restructured): the pair kernel (B = 32), the chunk
    # grid (B = 2), the fused query projection, multi-row cross-attention (prefill / beams), the fused self block and
    # the plain self-attention step at several lengths
    H, S, d = 20, 1500, 1280
    for B in (32, 2):
        k = torch.randn(B, H, S, 64, device="cuda", generator=g).bfloat16()
        v = torch.randn(B, H, S, 64, device="cuda", generator=g).bfloat16()
        for ql in (1, 4, 5):
            q = (torch.randn(B * ql, d, device="cuda", generator=g) * 0.3).bfloat16()
            o = torch.empty(B * ql, d, device="cuda", dtype=torch.bfloat16)
            ws = torch.zeros(ops.cross_attn_workspace_bytes(B, ql, H, 64, S) // 4 + 1, device="cuda")
            ops.cross_attn_step(q, B, ql, H, 64, k, v, S, o, ws)
            out[f"cross_B{B}_q{ql}"] = o.view(torch.int16).cpu().numpy()
        hbx = torch.randn(B, d, device="cuda", generator=g).bfloat16()
        Wq = (torch.randn(d, d, device="cuda", generator=g) / d ** 0.5).bfloat16()
        o = torch.empty(B, d, device="cuda", dtype=torch.bfloat16)
        ops.XqCrossPlan(hbx, ops.pack_weight(Wq), B, d, H, ln=(1e-5, ops.ln_colsum(Wq)),
                        bias=torch.randn(d, device="cuda", generator=g) * 0.1, scale=0.125, k=k, v=v, S=S, out=o,
                        workspace=torch.zeros(ops.xq_cross_workspace_bytes(B, d, H, S) // 4 + 1, device="cuda"))()
        out[f"xq_cross_B{B}"] = o.view(torch.int16).cpu().numpy()
        del k, v
        Wqkv = (torch.randn(3 * d, d, device="cuda", generator=g) / d ** 0.5).bfloat16()
        Wp3, cs3 = ops.pack_weight(Wqkv), ops.ln_colsum(Wqkv)
        b3 = torch.randn(3 * d, device="cuda", generator=g) * 0.1
        qkv = (torch.randn(B, 3 * d, device="cuda", generator=g) * 0.5).bfloat16()
        for t in (5, 100, 200):
            kc = torch.randn(B, H, 448, 64, device="cuda", generator=g).bfloat16()
            vc = torch.randn(B, H, 448, 64, device="cuda", generator=g).bfloat16()
            cur = torch.tensor([t], dtype=torch.int32, device="cuda")
            o = torch.empty(B, d, device="cuda", dtype=torch.bfloat16)
            ops.QkvSelfPlan(hbx, Wp3, B, d, H, ln=(1e-5, cs3), bias=b3, scale=0.125, k_cache=kc, v_cache=vc, t_max=448,
                            cur_len=cur, out=o,
                            workspace=torch.zeros(ops.qkv_self_workspace_bytes(B, d) // 4 + 1, device="cuda"))()
            out[f"qkv_self_B{B}_t{t}"] = o.view(torch.int16).cpu().numpy()
            o2 = torch.empty(B, d, device="cuda", dtype=torch.bfloat16)
            ops.self_attn_step(qkv, B, 1, H, 64, kc, vc, 448, cur, o2,
                               torch.zeros(ops.self_attn_workspace_bytes(B, H, 448) // 4 + 1, device="cuda"))
            out[f"self_attn_B{B}_t{t}"] = o2.view(torch.int16).cpu().numpy()
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
