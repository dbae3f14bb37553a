set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attn or attention or qkv_self or xq_cross or batch_invariant" --timeout 120 --timeout-method thread > gpurun_out/r03o_pytest_attn.log 2>&1 && echo ATTN_OK &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03o_bench.json 2> gpurun_out/r03o_bench.err && cat gpurun_out/r03o_bench.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03o_prof -o r03o -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03o_prof.log 2>&1 && echo PROF_OK &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -s > gpurun_out/r03o_pytest_gpu.log 2>&1 && echo ALL_OK
