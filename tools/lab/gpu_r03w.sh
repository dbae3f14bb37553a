set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03w_bench_prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r03w_bench_prof.log 2>&1 && echo PROF_OK &&
bash tools/pmc_only.sh r03w &&
timeout -k 10 600 python bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err && cat gpurun_out/r03w_bench.json
