# Round measurement set on the GPU box (tag $1): kernel-trace stats of the bench, FETCH / WRITE PMC passes over the
# decode kernels (tools/pmc_only.sh), their CSV summaries (rocpd databases stay on the box), then the bench line
# with its CPU baseline leg.   bash tools/lab/gpu_measure.sh r03ad
set -o pipefail
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${TAG}_bench_prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_prof.log 2>&1 && echo PROF_OK &&
python3 tools/rocpd_summary.py --stats /tmp/${TAG}_bench_prof/run_results.db gpurun_out/${TAG}_bench_kernel_stats.csv &&
bash tools/pmc_only.sh ${TAG} &&
python3 tools/rocpd_summary.py --pmc gpurun_out/${TAG}_pmc_fetch/run_results.db gpurun_out/${TAG}_pmc_fetch.csv &&
python3 tools/rocpd_summary.py --pmc gpurun_out/${TAG}_pmc_write/run_results.db gpurun_out/${TAG}_pmc_write.csv &&
rm -rf gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write &&
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && cat gpurun_out/${TAG}_bench.json
