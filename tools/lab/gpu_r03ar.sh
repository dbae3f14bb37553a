set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_configs.py --config 4 > gpurun_out/r03ar_config4.json 2> gpurun_out/r03ar_config4.err && cat gpurun_out/r03ar_config4.json
