#!/bin/bash
# Round-end check on the GPU box: GPU tests, smoke(), bench.py, the rocprofv3 passes, config 5.
#   bash tools/gpu_round_check.sh r01g   -> gpurun_out/<tag>_*
set -o pipefail
TAG=${1:-r01g}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 && echo SMOKE_OK &&
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && cat gpurun_out/${TAG}_bench.json &&
bash tools/profile.sh ${TAG} &&
timeout -k 10 200 python tools/bench_configs.py --config 5 --clips 64 > gpurun_out/${TAG}_config5.json 2> gpurun_out/${TAG}_config5.err && cat gpurun_out/${TAG}_config5.json
