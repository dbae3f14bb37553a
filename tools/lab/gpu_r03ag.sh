set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/lab/enc_split_streams.py > gpurun_out/r03ag_enc_split.txt 2>&1; rc=$?; cat gpurun_out/r03ag_enc_split.txt | grep -v amdgpu.ids; exit $rc
