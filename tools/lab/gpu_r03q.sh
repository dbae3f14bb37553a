set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KW_CROSS_ROW=0 timeout -k 10 300 python -u tools/kbench.py --only xq_cross,cross_attn --reps 20 > gpurun_out/r03q_kbench_row0.json 2>&1 && cat gpurun_out/r03q_kbench_row0.json &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "cross or xq_cross" --timeout 120 --timeout-method thread > gpurun_out/r03q_pytest_cross.log 2>&1 && echo CROSS_OK
