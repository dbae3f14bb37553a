set -e
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
KW_DEC_DBG=15 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_kb -o run -- python3 tools/kbench.py --only fc2_resid,o_resid,qkv_ln > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_lab -o run -- ./tools/lab/gemv_lab > /dev/null 2>&1
find gpurun_out/pf_kb gpurun_out/pf_lab -name "*kernel_stats.csv" | head
