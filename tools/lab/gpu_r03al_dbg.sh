set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/lab/replay_k_debug.py > gpurun_out/r03al_dbg.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03al_dbg.txt | tail -60; exit $rc
