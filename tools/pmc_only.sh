#!/bin/bash
# Only the two --pmc passes of tools/profile.sh (FETCH_SIZE, WRITE_SIZE over tools/kbench.py) plus the
# kernel-source hash they measured.   bash tools/pmc_only.sh r02f -> gpurun_out/<tag>_pmc_{fetch,write}
set -e
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ONLY=cross_attn,xq_cross,self_attn,qkv_self,o_resid,fc1_ln_gelu,fc2_resid,qkv_ln,xq_ln,lm_head
rm -rf gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 tools/kbench.py --eager --reps 2 --only $ONLY > gpurun_out/${TAG}_pmc_fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_write -o run -- python3 tools/kbench.py --eager --reps 2 --only $ONLY > gpurun_out/${TAG}_pmc_write.log 2>&1
python3 -c "import bench, json; print(json.dumps({'kernel_source_sha256': bench.kernel_source_hash()}))" > gpurun_out/${TAG}_pmc_fetch.meta.json
echo PMC_OK
