#!/usr/bin/env python
"""Decode-kernel microbenchmarks on the MI355X (development tool, not part of the product path).

Times each decode-step kernel at large-v3 shapes (B=32) cycling over 32 distinct weight / K-V
buffers (as the 32 decoder layers do) so the 256 MB Infinity Cache cannot serve repeats.

    python tools/kbench.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))

import torch  # noqa: E402

from kwhisper import ops  # noqa: E402


EAGER = False


def timeit(fns, reps):
    """Device time per launch: the launches are captured once into a hipGraph and replayed, so host
    launch overhead is excluded (kernel boundaries are included, as in the decode step)."""
    for f in fns:
        f()
    torch.cuda.synchronize()
    if EAGER:  # plain launches (for PMC passes: one counter record per dispatch)
        for _ in range(reps):
            for f in fns:
                f()
        torch.cuda.synchronize()
        return float("nan")
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(g, stream=side):
        for f in fns:
            f()
    torch.cuda.current_stream().wait_stream(side)
    g.replay()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        g.replay()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * len(fns))  # us per launch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--only", default="", help="comma list of kernel names to run (default: all)")
    ap.add_argument("--eager", action="store_true", help="no graph, no timing (for rocprofv3 --pmc passes)")
    ap.add_argument("--warm", action="store_true", help="one weight buffer per linear (L2/MALL-warm replays)")
    ap.add_argument("--self-t", default="132", help="comma list of self-attention lengths (cur_len) to time")
    ap.add_argument("--backend", default="torch", choices=("torch", "ctypes"),
                    help="ctypes: call the C ABI directly (with KWHISPER_LIB=<lab build> for geometry overrides)")
    a = ap.parse_args()
    ops.set_backend(a.backend)
    global EAGER
    EAGER = a.eager
    only = set(filter(None, a.only.split(",")))
    want = lambda n: not only or n in only  # noqa: E731
    dev = torch.device("cuda")
    B, d, H, S, F = 32, 1280, 20, 1500, 5120
    nl = a.layers
    res = {}
    hb = torch.randn(B, F, device=dev).bfloat16()
    h = torch.randn(B, d, device=dev)
    ws = torch.zeros(1 << 22, device=dev)
    for name, N, K, lna, resid in [("qkv_ln", 3 * d, d, True, False), ("o_resid", d, d, False, True),
                                   ("xq_ln", d, d, True, False), ("fc1_ln_gelu", F, d, True, False),
                                   ("fc2_resid", d, F, False, True), ("o_plain", d, d, False, False),
                                   ("lm_head", 51866, d, True, False)]:
        if not want(name):
            continue
        n_bufs = 1 if (name == "lm_head" or a.warm) else nl
        Ws = [ops.pack_weight((torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()) for _ in range(n_bufs)]
        cs = torch.zeros(N, device=dev)
        bias = torch.zeros(N, device=dev)
        C = torch.empty(B, N, device=dev) if name == "lm_head" else torch.empty(B, N, device=dev, dtype=torch.bfloat16)
        hr = torch.zeros(B, N, device=dev)
        hbr = torch.empty(B, N, device=dev, dtype=torch.bfloat16)
        plans = []
        for W in Ws:
            kw = dict(bias=bias, workspace=ws, ldx=F)
            if lna:
                kw["ln"] = (1e-5, cs)
            if resid:
                kw.update(resid=(hr, hbr, N, 0))
            else:
                kw["C"] = C
            if name.startswith("fc1"):
                kw["gelu"] = True
            plans.append(ops.DecLinearPlan(hb, W, B, N, K, **kw))
        us = timeit(plans, a.reps)
        res[name] = {"us": round(us, 2), "GBps": round(N * K * 2 / us / 1e3, 1)}
    # attention kernels (and the fused decode blocks: kw_dec_xq_cross, kw_dec_qkv_self)
    if not any(want(n) for n in ("cross_attn", "xq_cross", "self_attn", "qkv_self")):
        print(json.dumps(res))
        return
    q = torch.randn(B, d, device=dev).bfloat16()
    out = torch.empty(B, d, device=dev, dtype=torch.bfloat16)
    if want("cross_attn"):
        cross = [torch.randn(2, B, H, S, 64, device=dev).bfloat16() for _ in range(nl)]
        ws = torch.zeros(ops.cross_attn_workspace_bytes(B, 1, H, 64, S) // 4 + 1, device=dev)
        fns = [lambda c=c: ops.cross_attn_step(q, B, 1, H, 64, c[0], c[1], S, out, ws) for c in cross]
        us = timeit(fns, max(1, a.reps // 4))
        res["cross_attn"] = {"us": round(us, 2), "GBps": round(2 * B * H * S * 64 * 2 / us / 1e3, 1)}
        del cross
    if want("xq_cross"):  # the greedy step's cross block: LN-fused q projection + attention, per-layer K/V
        cross = [torch.randn(2, B, H, S, 64, device=dev).bfloat16() for _ in range(nl)]
        Wq = [ops.pack_weight((torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()) for _ in range(nl)]
        cs, bq = torch.zeros(d, device=dev), torch.zeros(d, device=dev)
        wsx = torch.zeros(ops.xq_cross_workspace_bytes(B, d, H, S) // 4 + 1, device=dev)
        hbd = hb[:, :d].contiguous()  # the engine's q = 1 residual mirror: [B][d]
        plans = [ops.XqCrossPlan(hbd, Wq[i], B, d, H, ln=(1e-5, cs), bias=bq, scale=0.125, k=cross[i][0], v=cross[i][1],
                                 S=S, out=out, workspace=wsx) for i in range(nl)]
        us = timeit(plans, max(1, a.reps // 4))
        res["xq_cross"] = {"us": round(us, 2), "GBps": round((2 * B * H * S * 64 * 2 + d * d * 2) / us / 1e3, 1)}
        del cross, Wq, plans
    if not want("self_attn") and not want("qkv_self"):
        print(json.dumps(res))
        return
    kc = torch.randn(nl, B, H, 448, 64, device=dev).bfloat16()
    vc = torch.randn(nl, B, H, 448, 64, device=dev).bfloat16()
    qkv = torch.randn(B, 3 * d, device=dev).bfloat16()
    sws = torch.zeros(ops.self_attn_workspace_bytes(B, H, 448) // 4 + 1, device=dev)
    for t in [int(x) for x in a.self_t.split(",")]:
        cur = torch.tensor([t], dtype=torch.int32, device=dev)
        fns = [lambda i=i, cur=cur: ops.self_attn_step(qkv, B, 1, H, 64, kc[i], vc[i], 448, cur, out, sws)
               for i in range(nl)]
        if want("self_attn"):
            res[f"self_attn_t{t}"] = {"us": round(timeit(fns, a.reps), 2)}
        if want("qkv_self"):  # the greedy step's self block: LN-fused qkv projection + attention + cache append
            Wqkv = [ops.pack_weight((torch.randn(3 * d, d, device=dev) / d ** 0.5).bfloat16()) for _ in range(nl)]
            cs3, b3 = torch.zeros(3 * d, device=dev), torch.zeros(3 * d, device=dev)
            qws = torch.zeros(ops.qkv_self_workspace_bytes(B, d) // 4 + 1, device=dev)
            hbd = hb[:, :d].contiguous()  # the engine's q = 1 residual mirror: [B][d]
            plans = [ops.QkvSelfPlan(hbd, Wqkv[i], B, d, H, ln=(1e-5, cs3), bias=b3, scale=0.125, k_cache=kc[i],
                                     v_cache=vc[i], t_max=448, cur_len=cur, out=out, workspace=qws)
                     for i in range(nl)]
            res[f"qkv_self_t{t}"] = {"us": round(timeit(plans, a.reps), 2)}
            del Wqkv, plans
    print(json.dumps(res))


if __name__ == "__main__":
    main()
