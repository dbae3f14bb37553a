set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attn or attention or qkv_self or xq_cross or batch_invariant" --timeout 120 --timeout-method thread > gpurun_out/r03t_pytest_attn.log 2>&1 && echo ATTN_OK &&
timeout -k 10 300 python -u tools/kbench.py --only qkv_self,self_attn,qkv_ln,xq_ln,xq_cross,cross_attn --self-t 1,64,132 --reps 20 > gpurun_out/r03t_kbench.json 2>&1 && cat gpurun_out/r03t_kbench.json &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03t_bench.json 2> gpurun_out/r03t_bench.err && cat gpurun_out/r03t_bench.json
