set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r01g_pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r01g_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench.py > gpurun_out/r01g_bench.json 2> gpurun_out/r01g_bench.err && cat gpurun_out/r01g_bench.json &&
bash tools/profile.sh r01g &&
timeout -k 10 200 python tools/bench_configs.py --config 5 --clips 64 > gpurun_out/r01g_config5.json 2> gpurun_out/r01g_config5.err && cat gpurun_out/r01g_config5.json
