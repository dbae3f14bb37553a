#!/bin/bash
# rocprofv3 passes behind profiles/ (run on the GPU box): kernel-trace stats of the bench, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes over the decode kernels (tools/kbench.py, eager).
# Each pass's rocpd database is reduced to a CSV (tools/rocpd_summary.py) and deleted, so what comes back
# under gpurun_out/ stays small (gpurun copies back at most 64 MiB).
#   bash tools/profile.sh r04 -> gpurun_out/<tag>_bench_kernel_stats.csv, <tag>_pmc_{fetch,write}.csv (+ .meta.json)
set -e
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RAW=/tmp/kw_prof_${TAG}
rm -rf "$RAW"
mkdir -p "$RAW"
ONLY=cross_attn,xq_cross,self_attn,qkv_self,o_resid,fc1_ln_gelu,fc2_resid,qkv_ln,xq_ln,lm_head
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$RAW/bench_prof" -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${TAG}_bench_prof.log 2>&1
python3 tools/rocpd_summary.py --stats "$RAW/bench_prof/run_results.db" gpurun_out/${TAG}_bench_kernel_stats.csv
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$RAW/pmc_fetch" -o run -- python3 tools/kbench.py --eager --reps 2 --only $ONLY > gpurun_out/${TAG}_pmc_fetch.log 2>&1
python3 tools/rocpd_summary.py --pmc "$RAW/pmc_fetch/run_results.db" gpurun_out/${TAG}_pmc_fetch.csv
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$RAW/pmc_write" -o run -- python3 tools/kbench.py --eager --reps 2 --only $ONLY > gpurun_out/${TAG}_pmc_write.log 2>&1
python3 tools/rocpd_summary.py --pmc "$RAW/pmc_write/run_results.db" gpurun_out/${TAG}_pmc_write.csv
# the kernel sources these counters measured (bench.py reports roofline.traffic only for the same sources)
python3 -c "import bench, json; print(json.dumps({'kernel_source_sha256': bench.kernel_source_hash()}))" > gpurun_out/${TAG}_pmc_fetch.meta.json
rm -rf "$RAW"
tail -1 gpurun_out/${TAG}_bench_prof.log
