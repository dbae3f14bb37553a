#!/usr/bin/env python
"""Per-kernel breakdown of ONE encoder pass from a rocprofv3 trace of bench.py (development tool).

Finds the last logmel_kernel dispatch in ``kernels`` (rocpd database), then lists the following kernels up to
the first decode linear, grouped by name with count / total / mean (us) and the share of the pass.

    python tools/enc_trace.py gpurun_out/<tag>_bench_prof/run_results.db
"""
import sqlite3
import sys


def main(path):
    db = sqlite3.connect(path)
    rows = [(n.replace("(anonymous namespace)::", "").replace("void ", ""), s, e)
            for n, s, e in db.execute("select name, start, end from kernels order by start")]
    idx = [i for i, r in enumerate(rows) if r[0].startswith("logmel_kernel")]
    i0 = idx[-1]
    seq = []
    for r in rows[i0:]:
        if "dec_linear" in r[0] or "embed_kernel" in r[0]:
            break
        seq.append(r)
    t0, t1 = seq[0][1], seq[-1][2]
    agg = {}
    for n, s, e in seq:
        k = n.split("(")[0][:60]
        c, tot = agg.get(k, (0, 0))
        agg[k] = (c + 1, tot + (e - s))
    busy = sum(v[1] for v in agg.values())
    print(f"encoder pass (log-mel .. cross-K/V): wall {(t1 - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, "
          f"gaps {(t1 - t0 - busy) / 1e3:.1f} us")
    for k, (c, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {k:60s} n={c:4d} total {tot / 1e3:9.1f} us  mean {tot / c / 1e3:8.1f} us  {100 * tot / busy:5.1f} %")
    # the encoder GEMMs in order within one layer (after the first attention)
    names = [r[0].split("(")[0] for r in seq]
    a = next(j for j, n in enumerate(names) if n.startswith("attn_fwd"))
    print("one layer:", [(names[j][:26], round((seq[j][2] - seq[j][1]) / 1e3, 1)) for j in range(a - 2, a + 6)])


if __name__ == "__main__":
    main(sys.argv[1])
