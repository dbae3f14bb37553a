# bench.py's N = 2 path rehearsed on one GPU: two ranks over gloo sharing cuda:0 (the driver's 8-GPU run uses RCCL)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp KW_BENCH_BACKEND=gloo
timeout -k 10 500 python bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03ap_bench_world2_gloo.json 2> gpurun_out/r03ap_bench_world2_gloo.err; rc=$?; cat gpurun_out/r03ap_bench_world2_gloo.json; tail -3 gpurun_out/r03ap_bench_world2_gloo.err; exit $rc
