set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attention" --timeout 120 --timeout-method thread > gpurun_out/r03u_pytest_attn.log 2>&1 && echo ATTN_OK &&
timeout -k 10 300 python -u tools/lab/enc_attn_ab.py > gpurun_out/r03u_enc_attn_ab.txt 2>&1 && cat gpurun_out/r03u_enc_attn_ab.txt
