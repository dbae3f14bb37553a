set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/lab/replay_k.py 2,4,8 > gpurun_out/r03am_replay_k.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03am_replay_k.txt | tail -14; exit $rc
