#!/bin/bash
# r06b: tail A/B (fused LM head + greedy step vs two launches) and a kernel trace of the fused bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/lab/tail_ab.py --rounds 3 > gpurun_out/r06b_tail_ab.txt 2>&1 && tail -2 gpurun_out/r06b_tail_ab.txt &&
RAW=/tmp/kw_prof_r06b && rm -rf $RAW && mkdir -p $RAW &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$RAW/bench_prof" -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r06b_bench_prof.log 2>&1 &&
python3 tools/rocpd_summary.py --stats "$RAW/bench_prof/run_results.db" gpurun_out/r06b_bench_kernel_stats.csv && head -20 gpurun_out/r06b_bench_kernel_stats.csv | cut -c1-150
