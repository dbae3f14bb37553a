set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "attn or qkv_self or xq_cross" --timeout 120 --timeout-method thread > gpurun_out/r03l_pytest_attn.log 2>&1 && echo ATTN_OK &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_generate.py -m gpu -x -q -s -k "fused" --timeout 200 --timeout-method thread > gpurun_out/r03l_pytest_fused.log 2>&1 && echo FUSED_OK &&
KW_CROSS_ROW=0 timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03l_bench_row0.json 2> gpurun_out/r03l_bench_row0.err && cat gpurun_out/r03l_bench_row0.json &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03l_bench.json 2> gpurun_out/r03l_bench.err && cat gpurun_out/r03l_bench.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03l_prof -o r03l -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03l_prof.log 2>&1 && echo PROF_OK
