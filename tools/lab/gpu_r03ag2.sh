set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/enc_parts_sweep.py > gpurun_out/r03ag_enc_parts.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03ag_enc_parts.txt | tail -8; [ $rc -eq 0 ] &&
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03ag_pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/r03ag_pytest_gpu.log; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03ag_bench.json 2> gpurun_out/r03ag_bench.err && cat gpurun_out/r03ag_bench.json
