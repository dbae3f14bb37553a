#!/usr/bin/env python
"""Lab (not product): kw_cross_attn_step of several builds of libkwhisper.so (ctypes, one process) on the same
inputs -- bitwise comparison -- and their timing over 32 layers' K/V.   python tools/lab/xa_dma_check.py A.so B.so [...]"""
import ctypes
import json
import sys

import torch


def load(path):
    lib = ctypes.CDLL(path)
    lib.kw_cross_attn_step.restype = ctypes.c_int
    lib.kw_cross_attn_step.argtypes = [ctypes.c_int, ctypes.c_void_p] + [ctypes.c_int64] * 4 + [ctypes.c_void_p] * 2 + \
        [ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    lib.kw_cross_attn_workspace.restype = ctypes.c_size_t
    lib.kw_cross_attn_workspace.argtypes = [ctypes.c_int64] * 5
    return lib


def main():
    paths = sys.argv[1:]
    libs = [load(p) for p in paths]
    import os
    B, H, S, hd, nl = int(os.environ.get("XA_B", 32)), 20, 1500, 64, 16
    QL = int(os.environ.get("XA_QLEN", 1))  # rows per item (beams: the MFMA kernel from 5)
    g = torch.Generator(device="cuda").manual_seed(0)
    cross = [torch.randn(2, B, H, S, hd, device="cuda", generator=g).bfloat16() for _ in range(nl)]
    q = (torch.randn(B * QL, H * hd, device="cuda", generator=g) * 2).bfloat16()
    wsb = libs[0].kw_cross_attn_workspace(B, QL, H, hd, S)
    res = {}
    outs = []
    s = torch.cuda.current_stream()
    for li, lib in enumerate(libs):
        ws = torch.zeros(wsb // 4 + 1, device="cuda")
        out = torch.empty(B * QL, H * hd, device="cuda", dtype=torch.bfloat16)

        def run(c):
            rc = lib.kw_cross_attn_step(1, q.data_ptr(), B, QL, H, hd, c[0].data_ptr(), c[1].data_ptr(), S,
                                        out.data_ptr(), ws.data_ptr(), wsb, s.cuda_stream)
            assert rc == 0
        run(cross[0])
        torch.cuda.synchronize()
        outs.append(out.clone())
        for _ in range(3):
            for c in cross:
                run(c)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            for c in cross:
                run(c)
        e1.record(s)
        e1.synchronize()
        res[paths[li]] = round(e0.elapsed_time(e1) * 1e3 / (10 * nl), 2)
    for li in range(1, len(libs)):
        res[f"{paths[li]} vs {paths[0]}"] = {"bitwise_equal": bool(torch.equal(outs[0], outs[li])),
                                             "max_abs_diff": float((outs[0].float() - outs[li].float()).abs().max())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
