set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -s --timeout 120 --timeout-method thread -k "cross_attn_enc or grouped" > gpurun_out/x11_kern.log 2>&1; echo kern rc $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_generate.py -x -q -s --timeout 200 --timeout-method thread -k "bf16_vs_reference or tiny_bf16_logits" > gpurun_out/x11_e2e.log 2>&1; echo e2e rc $?
for v in "" tools/lab/libkw_x1.so; do
  KWHISPER_LIB=$v timeout -k 10 60 python tools/lab/xenc_lab.py 2>&1 | grep us/launch
done
XSTAMPS=1 KWHISPER_LIB=tools/lab/libkw_xs.so timeout -k 10 60 python tools/lab/xenc_lab.py 2>&1 | grep -v amdgpu.ids | head -4
timeout -k 10 100 python tools/kbench.py --only xu,xv,xenc,o_resid 2>&1 | grep -v amdgpu.ids
