#!/usr/bin/env python
"""Lab (not product): per-workgroup s_memrealtime timeline of one kw_dec_chain launch (lab build with
-DKW_CH_STAMPS, KWHISPER_LIB pointing at it).  Large-v3 shapes, 32 rows; prints per phase the start, wait-done,
compute-done, epilogue and signal times (us after the first workgroup started; min / median / max)."""
from __future__ import annotations

import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "kotoba-whisper_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from kwhisper import _lib as L, ops
    lib = L.load()
    lib.kw_lab_chain_stamps.restype = ctypes.c_int
    dev = torch.device("cuda")
    d, ffn, M = 1280, 5120, 32
    g = torch.Generator(device="cpu").manual_seed(0)

    def w(n, k):
        t = (torch.randn((n, k), generator=g) * (k ** -0.5)).to(torch.bfloat16).to(dev)
        return ops.pack_weight(t), ops.ln_colsum(t)

    attn = torch.randn((M, d), generator=g).to(torch.bfloat16).to(dev)
    h = torch.randn((M, d), generator=g).to(dev)
    hb = h.to(torch.bfloat16)
    qx = torch.zeros((M, d), device=dev, dtype=torch.bfloat16)
    f = torch.zeros((M, ffn), device=dev, dtype=torch.bfloat16)
    ws = torch.zeros(((ops.dec_linear_workspace_bytes(d, ffn) + 3) // 4,), device=dev)
    sync = torch.zeros(((ops.dec_chain_sync_bytes() + 3) // 4,), device=dev, dtype=torch.int32)
    b = torch.zeros((ffn,), device=dev)
    lin = ops.DecLinearPlan
    sets = []
    for _ in range(8):  # distinct weights per launch (cold, as in a decode step)
        o_w, _ = w(d, d); xq_w, xq_cs = w(d, d); xo_w, _ = w(d, d); f1_w, f1_cs = w(ffn, d); f2_w, _ = w(d, ffn)
        sets.append(dict(
            o_xq=ops.DecChainPlan([lin(attn, o_w, M, d, d, bias=b[:d], resid=(h, hb, d, 0), workspace=ws, tag="o"),
                                   lin(hb, xq_w, M, d, d, ln=(1e-5, xq_cs), bias=b[:d], C=qx, workspace=ws, tag="xq")], sync),
            mlp=ops.DecChainPlan([lin(attn, xo_w, M, d, d, bias=b[:d], resid=(h, hb, d, 0), workspace=ws, tag="xo"),
                                  lin(hb, f1_w, M, ffn, d, ln=(1e-5, f1_cs), bias=b, C=f, gelu=True, workspace=ws),
                                  lin(f, f2_w, M, d, ffn, bias=b[:d], resid=(h, hb, d, 0), workspace=ws)], sync)))
    out = {}
    for name in ("o_xq", "mlp"):
        for s in sets:  # warm-up launches
            s[name]()
        torch.cuda.synchronize()
        reps = []
        for s in sets[:4]:
            s[name]()
            torch.cuda.synchronize()
            buf = (ctypes.c_ulonglong * (4096 * 8))()
            n = lib.kw_lab_chain_stamps(buf, 4096)
            st = np.frombuffer(buf, dtype=np.uint64)[: n * 8].reshape(n, 8).astype(np.int64)
            reps.append(st)
        plan = sets[0][name]
        offs = [0]
        for p in plan.plans:
            N, K = p.args.N, p.args.K
            offs.append(None)
        st = reps[-1]
        t0 = st[:, 0].min()
        rel = (st - t0) / 100.0  # 100 MHz ticks -> us
        rel[st == 0] = np.nan
        # phase ranges from the chain's own layout: recompute from kw geometry through the stamps' count
        out[name] = {"wgs": int(st.shape[0]), "rows": {}}
        bounds = {"o_xq": [80, 160], "mlp": [80, 240, 720]}[name]
        lo = 0
        for pi, hi in enumerate(bounds):
            seg = rel[lo:hi]
            out[name]["rows"][f"phase{pi}"] = {f"t{j}": [round(float(np.nanmin(seg[:, j])), 2), round(float(np.nanmedian(seg[:, j])), 2),
                                                          round(float(np.nanmax(seg[:, j])), 2)] for j in range(6)
                                               if not np.all(np.isnan(seg[:, j]))}
            lo = hi
        out[name]["end_us"] = round(float(np.nanmax(rel)), 2)
    print(json.dumps(out, indent=1))
    print("error flag", ops.dec_chain_status(sync))


if __name__ == "__main__":
    main()
