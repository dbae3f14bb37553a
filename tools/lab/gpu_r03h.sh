set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attn or qkv_self" --timeout 120 --timeout-method thread > gpurun_out/r03h_pytest_attn.log 2>&1 && echo ATTN_OK &&
timeout -k 10 200 python -u tools/kbench.py --only cross_attn,self_attn --reps 20 > gpurun_out/r03h_kbench.json 2>&1 && cat gpurun_out/r03h_kbench.json &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03h_bench.json 2> gpurun_out/r03h_bench.err && cat gpurun_out/r03h_bench.json &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h_pytest_gpu.log 2>&1 && echo ALL_OK
