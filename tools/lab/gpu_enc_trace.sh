# one encoder pass per kernel from a rocprofv3 trace of bench.py (tools/enc_trace.py), tag $1
set -o pipefail
TAG=${1:?tag}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/${TAG}_enc -o run -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 --kernel-iters 1 > gpurun_out/${TAG}_enc_trace_bench.log 2>&1 &&
python3 tools/enc_trace.py /tmp/${TAG}_enc/run_results.db > gpurun_out/${TAG}_enc_trace.txt 2>&1; cat gpurun_out/${TAG}_enc_trace.txt
