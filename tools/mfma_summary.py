#!/usr/bin/env python
"""Matrix-pipe utilisation per kernel from a rocprofv3 --pmc pass (development tool; the r02k method):

    cycles          = GRBM_GUI_ACTIVE / 8            (rocprofv3 sums the 8 XCDs)
    effective clock = cycles / kernel duration        (from the same pass's --kernel-trace)
    mfma busy       = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024 SIMDs)
    wave busy       = SQ_BUSY_CYCLES / cycles / 8     (per XCD, as a fraction of the active cycles)

    python tools/mfma_summary.py gpurun_out/<tag>_pmc_mfma/run_results.db profiles/<tag>_pmc_mfma_encoder.json "<source>"
"""
import json
import sqlite3
import sys


def main(db, out, source):
    c = sqlite3.connect(db)
    val = {}
    for kid, name, cn, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        val.setdefault((kid, name), {})[cn] = v
    dur = {}
    try:
        for kid, s, e in c.execute("select dispatch_id, start, end from kernels"):
            dur[kid] = e - s
    except sqlite3.Error:
        pass
    agg = {}
    for (kid, name), cs in val.items():
        a = agg.setdefault(name, {"n": 0, "gui": 0.0, "mfma": 0.0, "busy": 0.0, "ns": 0.0})
        a["n"] += 1
        a["gui"] += cs.get("GRBM_GUI_ACTIVE", 0.0)
        a["mfma"] += cs.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a["busy"] += cs.get("SQ_BUSY_CYCLES", 0.0)
        a["ns"] += dur.get(kid, 0.0)
    rows = []
    for name, a in sorted(agg.items(), key=lambda kv: -kv[1]["gui"]):
        cyc = a["gui"] / 8 / a["n"]
        rows.append({"kernel": name[:160], "dispatches": a["n"], "avg_us": round(a["ns"] / a["n"] / 1e3, 1) if a["ns"] else None,
                     "grbm_gui_active_per_xcd": round(cyc),
                     "effective_clock_ghz": round(cyc / (a["ns"] / a["n"]), 3) if a["ns"] else None,
                     "mfma_busy_frac": round(a["mfma"] / a["n"] / (cyc * 1024), 3) if cyc else None})
    with open(out, "w") as f:
        json.dump({"source": source, "formulas": __doc__.split("\n\n")[1].strip(), "kernels": rows}, f, indent=1)
    for r in rows[:12]:
        print(r)


if __name__ == "__main__":
    main(*sys.argv[1:4])
