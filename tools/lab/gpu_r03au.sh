# r03au lab: cross block after a partial default-policy pre-read of its K/V (Infinity Cache residency)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 180 python -u tools/lab/mall_prefetch.py > gpurun_out/r03au_mall_prefetch.txt 2>&1; rc=$?; cat gpurun_out/r03au_mall_prefetch.txt; exit $rc
