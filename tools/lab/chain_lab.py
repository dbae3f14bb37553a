#!/usr/bin/env python
"""Lab (not product): kw_dec_chain vs the same decode linears launched one by one (large-v3 shapes, B = 32).

32 layers of random packed weights (distinct buffers, as in a decode step); per layer the (o -> cross q) and
(cross o -> fc1 -> fc2) runs.  Checks the chained results bitwise against the separate launches, then times
both as captured graphs (all 32 layers per replay).

    python tools/lab/chain_lab.py [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--layers", type=int, default=32)
    ap.add_argument("--rows", type=int, default=32)
    a = ap.parse_args()
    from kwhisper import ops
    dev = torch.device("cuda")
    d, ffn, M, Lk = 1280, 5120, a.rows, a.layers
    g = torch.Generator(device="cpu").manual_seed(0)

    def w(n, k):
        t = (torch.randn((n, k), generator=g) * (k ** -0.5)).to(torch.bfloat16)
        return ops.pack_weight(t.to(dev)), ops.ln_colsum(t.to(dev))

    def b(n):
        return (torch.randn((n,), generator=g) * 0.1).to(dev)

    layers = []
    for _ in range(Lk):
        o_w, _ = w(d, d)
        xq_w, xq_cs = w(d, d)
        xo_w, _ = w(d, d)
        f1_w, f1_cs = w(ffn, d)
        f2_w, _ = w(d, ffn)
        layers.append(dict(o_w=o_w, o_b=b(d), xq_w=xq_w, xq_cs=xq_cs, xq_b=b(d), xo_w=xo_w, xo_b=b(d),
                           f1_w=f1_w, f1_cs=f1_cs, f1_b=b(ffn), f2_w=f2_w, f2_b=b(d)))
    attn = (torch.randn((M, d), generator=g)).to(torch.bfloat16).to(dev)
    h0 = torch.randn((M, d), generator=g).to(dev)
    ws = torch.zeros(((ops.dec_linear_workspace_bytes(d, ffn) + 3) // 4,), device=dev)
    sync = torch.zeros(((ops.dec_chain_sync_bytes() + 3) // 4,), device=dev, dtype=torch.int32)

    def bufs():
        h = h0.clone()
        return dict(h=h, hb=h.to(torch.bfloat16), qx=torch.zeros((M, d), device=dev, dtype=torch.bfloat16),
                    ffn=torch.zeros((M, ffn), device=dev, dtype=torch.bfloat16))

    def plans(bf, chained, part="all"):
        seq = []
        lin = ops.DecLinearPlan
        for L in layers:
            a1 = [lin(attn, L["o_w"], M, d, d, bias=L["o_b"], resid=(bf["h"], bf["hb"], d, 0), workspace=ws, tag="o"),
                  lin(bf["hb"], L["xq_w"], M, d, d, ln=(1e-5, L["xq_cs"]), bias=L["xq_b"], C=bf["qx"], scale=0.125,
                      scale_cols=d, workspace=ws, tag="xq")]
            a2 = [lin(attn, L["xo_w"], M, d, d, bias=L["xo_b"], resid=(bf["h"], bf["hb"], d, 0), workspace=ws, tag="xo"),
                  lin(bf["hb"], L["f1_w"], M, ffn, d, ln=(1e-5, L["f1_cs"]), bias=L["f1_b"], C=bf["ffn"], gelu=True,
                      workspace=ws, tag="fc1"),
                  lin(bf["ffn"], L["f2_w"], M, d, ffn, bias=L["f2_b"], resid=(bf["h"], bf["hb"], d, 0), workspace=ws,
                      tag="fc2")]
            a1 = a1 if part in ("all", "o_xq") else []
            a2 = a2 if part in ("all", "mlp") else []
            if chained:
                seq += ([ops.DecChainPlan(a1, sync)] if a1 else []) + ([ops.DecChainPlan(a2, sync)] if a2 else [])
            else:
                seq += a1 + a2
        return seq

    res = {}
    bs, bc = bufs(), bufs()
    ps, pc = plans(bs, False), plans(bc, True)
    for p in ps:
        p()
    for p in pc:
        p()
    torch.cuda.synchronize()
    res["chain_error_flag"] = ops.dec_chain_status(sync)
    res["bitwise"] = {k: bool(torch.equal(bs[k], bc[k])) for k in bs}
    res["max_abs_h"] = float((bs["h"] - bc["h"]).abs().max())
    print(json.dumps(res), flush=True)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    times = {}
    runs = [("separate", ps), ("chained", pc)]
    for part in ("o_xq", "mlp"):
        runs += [(part + "_separate", plans(bs, False, part)), (part + "_chained", plans(bc, True, part))]
    for name, seq in runs:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            for p in seq:  # warm (and first-touch) outside the capture
                p()
            torch.cuda.synchronize()
            with torch.cuda.graph(graph, stream=s):
                for p in seq:
                    p()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        graph.replay()
        e0.record()
        for _ in range(a.iters):
            graph.replay()
        e1.record()
        e1.synchronize()
        times[name] = round(e0.elapsed_time(e1) * 1e3 / a.iters / Lk, 2)
        del graph
    res["us_per_layer (o,xq,xo,fc1,fc2)"] = times
    res["chain_error_flag_after"] = ops.dec_chain_status(sync)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
