set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/enc_attn_l2_ab.py > gpurun_out/r03x_enc_attn_ab.txt 2>&1; rc=$?; cat gpurun_out/r03x_enc_attn_ab.txt; [ $rc -eq 0 ] &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attention" > gpurun_out/r03x_pytest_attn.txt 2>&1; rc=$?; tail -3 gpurun_out/r03x_pytest_attn.txt; [ $rc -eq 0 ] &&
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r03x_bench.json 2> gpurun_out/r03x_bench.err && cat gpurun_out/r03x_bench.json
