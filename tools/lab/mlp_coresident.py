#!/usr/bin/env python
"""Lab driver (not product): the fused decode feed-forward block kw_dec_mlp against the two kw_dec_linear launches.

The fused block lost in rounds 4 and 5 (profiles/r05b_mlp_decomposition.txt), so libkwhisper.so no longer carries
it; the kernel lives in tools/lab/lab_switches.diff (behind KW_LAB_MLP once applied).  Build a lab library and point
this at it:

    bash tools/lab/mlp_lab_build.sh "-DKW_LAB_MLP"
    KWHISPER_LIB=$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so \\
    KWHISPER_TORCH_LIB=$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_torch_lab.so \\
         python tools/lab/mlp_coresident.py [--check] [--reps 40]

--check: h within f32 summation order of the two launches (fc1 is dec_linear's arithmetic; fc2 sums K in its own
5-k-tile slices), the flags re-armed after every launch, and the fault-injection word turning one launch's rows NaN.
Timing: 32 distinct weight buffers (the 32 decoder layers) replayed from a hipGraph, B = 32, d 1280, F 5120.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "kotoba-whisper_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

from kwhisper import _lib as L, ops  # noqa: E402

c_vp, c_i64 = ctypes.c_void_p, ctypes.c_int64


class MlpArgs(ctypes.Structure):  # tools/lab/kw_mlp_lab.h kw_dec_mlp_args
    _fields_ = [
        ("x", c_vp), ("ldx", c_i64), ("ln_eps", ctypes.c_float), ("fc1_colsum", c_vp), ("fc1_w", c_vp),
        ("fc1_bias", c_vp), ("fc2_w", c_vp), ("fc2_bias", c_vp), ("h", c_vp), ("hb", c_vp), ("ldh", c_i64),
        ("M", c_i64), ("d", c_i64), ("F", c_i64), ("workspace", c_vp), ("ws_bytes", ctypes.c_size_t),
    ]


def lab_lib():
    lib = L.lib()
    if not hasattr(lib, "kw_dec_mlp"):
        raise SystemExit("KWHISPER_LIB is not a KW_LAB_MLP build (kw_dec_mlp missing)")
    lib.kw_dec_mlp.restype, lib.kw_dec_mlp.argtypes = ctypes.c_int, [ctypes.POINTER(MlpArgs), c_vp]
    for f in ("kw_dec_mlp_workspace", "kw_dec_mlp_status_offset"):
        getattr(lib, f).restype, getattr(lib, f).argtypes = ctypes.c_size_t, [c_i64, c_i64, c_i64]
    lib.kw_dec_mlp_supported.restype, lib.kw_dec_mlp_supported.argtypes = ctypes.c_int, [c_i64, c_i64, c_i64]
    return lib


def mlp_call(lib, h, hb, W1, W2, M, d, F, eps, cs1, b1, b2, ws):
    a = MlpArgs(hb.data_ptr(), d, eps, cs1.data_ptr(), W1.data_ptr(), b1.data_ptr(), W2.data_ptr(), b2.data_ptr(),
                h.data_ptr(), hb.data_ptr(), d, M, d, F, ws.data_ptr(), ws.numel() * 4)
    keep = (a, h, hb, W1, W2, cs1, b1, b2, ws)

    def run():
        L.check(lib.kw_dec_mlp(ctypes.byref(keep[0]), c_vp(torch.cuda.current_stream().cuda_stream)), "kw_dec_mlp")
    return run


def check(lib, M, d, F):
    eps = 1e-5
    torch.manual_seed(M + 11)
    W1 = (torch.randn(F, d, device="cuda") / d ** 0.5).bfloat16()
    W2 = (torch.randn(d, F, device="cuda") / F ** 0.5).bfloat16()
    p1, cs1, p2 = ops.pack_weight(W1), ops.ln_colsum(W1), ops.pack_weight(W2)
    b1, b2 = torch.randn(F, device="cuda") * 0.1, torch.randn(d, device="cuda") * 0.1
    lws = torch.zeros(max(ops.dec_linear_workspace_bytes(F, d), ops.dec_linear_workspace_bytes(d, F)) // 4 + 1,
                      device="cuda")
    ws = torch.zeros(lib.kw_dec_mlp_workspace(M, d, F) // 4, device="cuda")
    st = lib.kw_dec_mlp_status_offset(M, d, F) // 4
    worst = 0.0
    for rep in range(4):
        h0 = torch.randn(M, d, device="cuda") * 2
        hb0 = h0.bfloat16()
        h1, hb1 = h0.clone(), hb0.clone()
        ffn = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
        ops.DecLinearPlan(hb1, p1, M, F, d, ln=(eps, cs1), bias=b1, C=ffn, gelu=True, workspace=lws)()
        ops.DecLinearPlan(ffn, p2, M, d, F, bias=b2, resid=(h1, hb1, d, 0), workspace=lws)()
        h2, hb2 = h0.clone(), hb0.clone()
        if rep == 2:
            ws.view(torch.int32)[st + 1] = 1  # fault injection: fc1 workgroup 0 skips its flag once
        mlp_call(lib, h2, hb2, p1, p2, M, d, F, eps, cs1, b1, b2, ws)()
        torch.cuda.synchronize()
        head = ws.view(torch.int32)[:1024]
        if rep == 2:
            assert int(head[st]) != 0 and bool(torch.isnan(h2).any(dim=1).all()), "the dropped flag did not time out"
            ws.zero_()
            continue
        assert int(head.abs().sum()) == 0, "flags not re-armed / a poll timed out"
        err = (h2 - h1).abs().max().item()
        worst = max(worst, err)
        assert err <= 2e-5 * (1 + h1.abs().max().item()), (rep, err)
        assert torch.equal(hb2, h2.bfloat16())
    return worst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--reps", type=int, default=40)
    a = ap.parse_args()
    import kbench

    lib = lab_lib()
    out = {}
    if a.check:
        out["check_max_abs_diff"] = {f"{M}x{d}x{F}": check(lib, M, d, F)
                                     for M, d, F in ((32, 1280, 5120), (7, 1280, 5120), (1, 1280, 5120), (5, 384, 1536))}
    dev = torch.device("cuda")
    B, d, F, nl = 32, 1280, 5120, 32
    W1 = [ops.pack_weight((torch.randn(F, d, device=dev) / d ** 0.5).bfloat16()) for _ in range(nl)]
    W2 = [ops.pack_weight((torch.randn(d, F, device=dev) / F ** 0.5).bfloat16()) for _ in range(nl)]
    cs1, b1, b2 = torch.zeros(F, device=dev), torch.zeros(F, device=dev), torch.zeros(d, device=dev)
    hm, hbm = torch.zeros(B, d, device=dev), torch.zeros(B, d, device=dev, dtype=torch.bfloat16)
    wsm = torch.zeros(lib.kw_dec_mlp_workspace(B, d, F) // 4, device=dev)
    fns = [mlp_call(lib, hm, hbm, W1[i], W2[i], B, d, F, 1e-5, cs1, b1, b2, wsm) for i in range(nl)]
    us = kbench.timeit(fns, a.reps)
    out["mlp"] = {"us": round(us, 2), "GBps": round(2 * F * d * 2 / us / 1e3, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
