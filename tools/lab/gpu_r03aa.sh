set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r03aa_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r03aa_pytest_gpu.log; [ $rc -eq 0 ] && echo TESTS_OK &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03aa_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench.py > gpurun_out/r03aa_bench.json 2> gpurun_out/r03aa_bench.err && cat gpurun_out/r03aa_bench.json
