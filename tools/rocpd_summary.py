#!/usr/bin/env python
"""Turn rocprofv3 rocpd databases (gpurun_out/<run>/run_results.db) into the small CSV summaries kept
under profiles/ (development tool).

    python tools/rocpd_summary.py --stats gpurun_out/r01_bench_prof/run_results.db profiles/r01_bench_kernel_stats.csv
    python tools/rocpd_summary.py --pmc gpurun_out/r01_pmc_fetch/run_results.db profiles/r01_pmc_fetch.csv

``--stats``: per kernel calls / total / average / min / max duration (ns) and share of GPU time, the
rocprofv3 ``--stats`` table.  ``--pmc``: per kernel and counter the dispatch count and mean / min /
max value as rocprofv3 reports it (FETCH_SIZE / WRITE_SIZE in KB; no correction applied here).
"""
from __future__ import annotations

import argparse
import csv
import re
import sqlite3


def _short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name if len(name) <= 160 else name[:157] + "..."


def stats(db: str, out: str) -> None:
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
                          "from kernels group by name order by sum(end-start) desc"))
    tot = sum(r[2] for r in rows) or 1
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
        for n, k, s, a, mn, mx in rows:
            w.writerow([_short(n), k, s, round(a, 1), mn, mx, round(100.0 * s / tot, 3)])


def pmc(db: str, out: str) -> None:
    c = sqlite3.connect(db)
    rows = list(c.execute("select kernel_name, counter_name, count(*), avg(value), min(value), max(value) "
                          "from counters_collection group by kernel_name, counter_name order by kernel_name"))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Counter", "Dispatches", "Mean", "Min", "Max"])
        for n, cn, k, a, mn, mx in rows:
            w.writerow([_short(n), cn, k, round(a, 3), mn, mx])


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    g = ap.add_mutually_exclusive_group(required=True)
    g.add_argument("--stats", action="store_true")
    g.add_argument("--pmc", action="store_true")
    ap.add_argument("db")
    ap.add_argument("out")
    a = ap.parse_args()
    (stats if a.stats else pmc)(a.db, a.out)
