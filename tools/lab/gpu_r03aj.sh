set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_generate.py -k "streams" > gpurun_out/r03aj_pytest.txt 2>&1; rc=$?; tail -8 gpurun_out/r03aj_pytest.txt; [ $rc -eq 0 ] &&
timeout -k 10 300 python -u tools/lab/prefill_split.py > gpurun_out/r03aj_prefill_split.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03aj_prefill_split.txt | tail -3; exit $rc
