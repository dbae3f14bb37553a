set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/lab/prefill_split.py > gpurun_out/r03ah_prefill_split.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03ah_prefill_split.txt | tail -14; exit $rc
