# config 4 (320 clips) under a kernel trace: GPU busy time vs the loop's wall time (the trace's last `seconds`)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/r03as -o run -- python3 tools/bench_configs.py --config 4 --n-clips 320 > gpurun_out/r03as_config4_prof.json 2> gpurun_out/r03as_config4_prof.err && cat gpurun_out/r03as_config4_prof.json &&
python3 - <<'PY'
import json, sqlite3, collections
secs = json.load(open("gpurun_out/r03as_config4_prof.json"))["seconds"]
c = sqlite3.connect("/tmp/r03as/run_results.db")
rows = list(c.execute("select start, end, name from kernels order by start"))
t1 = max(e for _, e, _ in rows)
w0 = t1 - int(secs * 1e9)
rows = [r for r in rows if r[0] >= w0]
busy = 0; last_end = None; gaps = []
for s, e, n in rows:
    if last_end is not None and s > last_end:
        gaps.append((s - last_end, n, prev))
    busy += e - s
    last_end = max(last_end or e, e); prev = n
span = t1 - w0
print(f"timed window {span/1e6:.1f} ms: kernels busy {busy/1e6:.1f} ms ({100*busy/span:.1f} %); "
      f"gaps > 50 us {sum(g for g, _, _ in gaps if g > 50000)/1e6:.1f} ms in {sum(1 for g, _, _ in gaps if g > 50000)}")
big = collections.Counter()
for g, n, p in gaps:
    if g > 50000:
        big[(p.split('(')[0][:40], n.split('(')[0][:40])] += g
for (p, n), g in big.most_common(8):
    print(f"  {g/1e6:8.1f} ms  after {p}  before {n}")
PY
