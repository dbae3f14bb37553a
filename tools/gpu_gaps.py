#!/usr/bin/env python
"""GPU idle gaps from a rocprofv3 database (development tool): kernels sorted by start; prints the
largest gaps between one kernel's end and the next kernel's start, with the kernels on either side.

    python tools/gpu_gaps.py gpurun_out/<run>/run_results.db [--top 15] [--min-us 20]
"""
import argparse
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=15)
ap.add_argument("--min-us", type=float, default=20.0)
ap.add_argument("--window", default=None, help="NAME:i:j -- only between the i-th and j-th start of a kernel "
                                                "whose name contains NAME (e.g. logmel_kernel:2:3 = bench's timed step)")
a = ap.parse_args()
rows = sqlite3.connect(a.db).execute("select start, end, name from kernels order by start").fetchall()
if a.window:
    name, i, j = a.window.split(":")
    marks = [r[0] for r in rows if name in r[2]]
    lo, hi_ = marks[int(i) - 1], marks[int(j) - 1] if int(j) <= len(marks) else float("inf")
    rows = [r for r in rows if lo <= r[0] < hi_]
gaps = []
hi = rows[0][1]
prev = rows[0][2]
for s, e, n in rows[1:]:
    if s > hi:
        gaps.append(((s - hi) / 1e3, prev[:60], n[:60]))
    if e > hi:
        hi, prev = e, n
span = (max(r[1] for r in rows) - rows[0][0]) / 1e3
big = [g for g in gaps if g[0] >= a.min_us]
print(f"kernels {len(rows)}, span {span / 1e3:.1f} ms, idle {sum(g[0] for g in gaps) / 1e3:.1f} ms "
      f"(gaps >= {a.min_us} us: {len(big)}, {sum(g[0] for g in big) / 1e3:.1f} ms)")
for g in sorted(gaps, reverse=True)[: a.top]:
    print(f"{g[0]:10.1f} us  after {g[1]!r:62s} before {g[2]!r}")
