#!/usr/bin/env python
"""kw_dec_oxq_cross vs its two launches (lab r05z): large-v3 greedy step shapes (M = 32, d = 1280, H = 20, S = 1500),
32 distinct layers' weights and K / V cycled in a captured graph (tools/kbench.py's timeit)."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from kwhisper import ops  # noqa: E402
from kbench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    M, d, H, S, nl = 32, 1280, 20, 1500, int(sys.argv[1]) if len(sys.argv) > 1 else 32
    eps = 1e-5
    attn = torch.randn(M, d, device=dev).bfloat16()
    h = torch.randn(M, d, device=dev)
    hb = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
    layers = []
    for _ in range(nl):
        Wo = (torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()
        Wq = (torch.randn(d, d, device=dev) / d ** 0.5).bfloat16()
        layers.append(dict(po=ops.pack_weight(Wo), bo=torch.zeros(d, device=dev), pq=ops.pack_weight(Wq),
                           cs=ops.ln_colsum(Wq), bq=torch.zeros(d, device=dev),
                           k=torch.randn(M, H, S, 64, device=dev).bfloat16(),
                           v=torch.randn(M, H, S, 64, device=dev).bfloat16()))
    lws = torch.zeros(ops.dec_linear_workspace_bytes(d, d) // 4 + 1, device=dev)
    xws = torch.zeros(ops.xq_cross_workspace_bytes(M, d, H, S) // 4 + 1, device=dev)
    ows = torch.zeros(ops.oxq_cross_workspace_bytes(M, d, H, S) // 4 + 1, device=dev)
    res = {}
    o_only = [ops.DecLinearPlan(attn, L["po"], M, d, d, bias=L["bo"], resid=(h, hb, d, 0), workspace=lws) for L in layers]
    xq_only = [ops.XqCrossPlan(hb, L["pq"], M, d, H, ln=(eps, L["cs"]), bias=L["bq"], scale=0.125, k=L["k"], v=L["v"],
                               S=S, out=attn, workspace=xws) for L in layers]
    two = [f for pair in zip(o_only, xq_only) for f in pair]
    fused = [ops.OxqCrossPlan(attn, L["po"], L["bo"], h, hb, M, d, H, W=L["pq"], ln=(eps, L["cs"]), bias=L["bq"],
                              scale=0.125, k=L["k"], v=L["v"], S=S, out=attn, workspace=ows) for L in layers]
    res["o_us"] = round(timeit(o_only, 10), 2)
    res["xq_cross_us"] = round(timeit(xq_only, 10), 2)
    res["o+xq_cross_us_per_layer"] = round(2 * timeit(two, 10), 2)
    res["oxq_cross_us"] = round(timeit(fused, 10), 2)
    torch.cuda.synchronize()
    res["status_words_zero"] = int(ows.view(torch.int32).abs().sum()) == 0
    print(json.dumps(res))


if __name__ == "__main__":
    main()
