set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "cross_attn" --timeout 120 --timeout-method thread > gpurun_out/r03d_pytest_cross.log 2>&1 && echo CROSS_OK &&
timeout -k 10 200 python -u tools/kbench.py --only cross_attn --reps 20 > gpurun_out/r03d_kbench.json 2>&1 && cat gpurun_out/r03d_kbench.json &&
timeout -k 10 200 python -u tools/lab/xa_lab.py > gpurun_out/r03d_xa_lab.log 2>&1 && head -3 gpurun_out/r03d_xa_lab.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_generate.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest_gen.log 2>&1 && echo GEN_OK &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.err && cat gpurun_out/r03d_bench.json
