set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/c4_probe.py > gpurun_out/r03a_c4_probe.log 2>&1 && echo PROBE_OK &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03a_pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err && cat gpurun_out/r03a_bench.json
