# Round-end measurement set (tag $1): GPU tests, smoke, bench line (CPU baseline leg), bench kernel trace,
# config 4 (1768-clip stand-in) and config 5 (64 windows).  PMC passes: tools/lab/gpu_measure.sh.
set -o pipefail
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] && echo TESTS_OK &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && cat gpurun_out/${TAG}_bench.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${TAG}_bench_prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_prof.log 2>&1 && echo PROF_OK &&
python3 tools/rocpd_summary.py --stats /tmp/${TAG}_bench_prof/run_results.db gpurun_out/${TAG}_bench_kernel_stats.csv &&
timeout -k 10 300 python tools/bench_configs.py --config 4 > gpurun_out/${TAG}_config4.json 2> gpurun_out/${TAG}_config4.err && cat gpurun_out/${TAG}_config4.json &&
timeout -k 10 300 python tools/bench_configs.py --config 5 --clips 64 > gpurun_out/${TAG}_config5.json 2> gpurun_out/${TAG}_config5.err && cat gpurun_out/${TAG}_config5.json
