#!/usr/bin/env python
"""Encoder kernel timeline from a rocprofv3 kernel-trace CSV (development tool, lab r05o).

Reads ``<dir>/run_kernel_trace.csv`` of ``tools/enc_pass.py`` and prints, for the LAST encoder pass (the passes are
cut at gaps > 1 ms): the wall time, the time at least one kernel runs (union of intervals), the time two run at once,
and per kernel family the launches, the summed duration and the mean.

    python tools/lab/enc_timeline.py gpurun_out/r05o_s2/run_kernel_trace.csv
"""
from __future__ import annotations

import csv
import json
import re
import sys


def family(name: str) -> str:
    for pat, fam in [(r"gemm256_kernel<2", "gemm_headsplit"), (r"gemm256_kernel<0", "gemm_store"),
                     (r"gemm256_kernel<1", "gemm_resid"), (r"attn_fwd", "attention"), (r"layernorm", "layernorm"),
                     (r"gemm_bf16_kernel", "gemm128"), (r"mel_tm|conv", "stem")]:
        if re.search(pat, name):
            return fam
    return name[:40]


def main(path: str) -> None:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # split into passes at host gaps > 1 ms
    passes, cur, last_end = [], [], None
    for s, e, n in rows:
        if last_end is not None and s - last_end > 1_000_000:
            passes.append(cur)
            cur = []
        cur.append((s, e, n))
        last_end = max(last_end or e, e)
    passes.append(cur)
    p = passes[-1]
    t0, t1 = p[0][0], max(e for _, e, _ in p)
    ev = sorted([(s, 1) for s, _, _ in p] + [(e, -1) for _, e, _ in p])
    busy = both = 0
    depth, prev = 0, t0
    for t, d in ev:
        if depth >= 1:
            busy += t - prev
        if depth >= 2:
            both += t - prev
        depth += d
        prev = t
    fams = {}
    for s, e, n in p:
        f = fams.setdefault(family(n), [0, 0])
        f[0] += 1
        f[1] += e - s
    out = {"passes": len(passes), "kernels": len(p), "wall_ms": round((t1 - t0) / 1e6, 3),
           "busy_ms": round(busy / 1e6, 3), "idle_ms": round((t1 - t0 - busy) / 1e6, 3),
           "overlap_ms": round(both / 1e6, 3),
           "families": {k: {"n": v[0], "sum_ms": round(v[1] / 1e6, 3), "mean_us": round(v[1] / v[0] / 1e3, 1)}
                        for k, v in sorted(fams.items(), key=lambda kv: -kv[1][1])}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
