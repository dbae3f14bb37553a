set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/lab/enc_ratio_sweep.py > gpurun_out/r03aq_enc_ratio.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03aq_enc_ratio.txt | tail -6; exit $rc
