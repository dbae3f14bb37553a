#!/bin/bash
# Kernel trace of the config-4 loop (320 stand-in clips, timestamps, gather at the end) on the final tree, reduced to a
# per-kernel CSV (the rocpd database is deleted: gpurun copies back at most 64 MiB).
#   bash tools/prof_config4.sh r04y -> gpurun_out/<tag>_config4_kernel_stats.csv, <tag>_config4_prof.log
set -e
TAG=${1:-r04}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RAW=/tmp/kw_c4prof_${TAG}
rm -rf "$RAW"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$RAW" -o run -- python3 tools/bench_configs.py --config 4 --n-clips 320 > gpurun_out/${TAG}_config4_prof.log 2>&1
python3 tools/rocpd_summary.py --stats "$RAW/run_results.db" gpurun_out/${TAG}_config4_kernel_stats.csv
rm -rf "$RAW"
echo C4PROF_OK
