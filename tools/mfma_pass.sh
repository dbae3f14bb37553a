#!/bin/bash
# One matrix-pipe counter pass over the one-pass encoder (tools/enc_pass.py --streams 1), reduced to a JSON summary
# per kernel (tools/mfma_summary.py) and the rocpd database deleted (gpurun copies back at most 64 MiB).
#   bash tools/mfma_pass.sh r04j -> gpurun_out/<tag>_pmc_mfma_encoder.json
set -e
TAG=${1:-r04}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RAW=/tmp/kw_mfma_${TAG}
rm -rf "$RAW"
timeout -k 10 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$RAW" -o run -- python3 tools/enc_pass.py --streams 1 > gpurun_out/${TAG}_pmc_mfma.log 2>&1
python3 tools/mfma_summary.py "$RAW/run_results.db" gpurun_out/${TAG}_pmc_mfma_encoder.json "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace over tools/enc_pass.py --streams 1 (large-v3, B = 32)"
rm -rf "$RAW"
echo MFMA_OK
