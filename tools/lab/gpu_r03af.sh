set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu tests/test_gpu_generate.py tests/test_gpu_workloads.py -k "bf16_beam or config5_pipeline_kotoba_bf16" > gpurun_out/r03af_pytest.txt 2>&1; rc=$?; grep -E "tiny bf16|config5 bf16|passed|failed|Error" gpurun_out/r03af_pytest.txt | tail -30; exit $rc
