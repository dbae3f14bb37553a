set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -k "cross_attn_enc or grouped" > gpurun_out/x6_kern.log 2>&1; echo kern rc $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_generate.py -x -q -s --timeout 200 --timeout-method thread -k "bf16" > gpurun_out/x6_e2e.log 2>&1; echo e2e rc $?
