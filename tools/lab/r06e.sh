#!/bin/bash
# r06e: bf16 multi-pass tendency scan over numpy-recipe seeds (candidates for the fp32 scan), then the chain stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/lab/chain_stamps.bin > gpurun_out/r06e_chain_stamps.txt 2>&1; echo "stamps rc=$?"
for SEED in ${SEEDS:-2 3 4 5 6 7 8 9}; do
  timeout -k 10 150 python -u tools/find_multipass.py --weights numpy --seed $SEED --dtype bfloat16 --n-clips 1768 \
    --stop-after 4 --out gpurun_out/r06e_multipass_bf16_s$SEED.json > gpurun_out/r06e_scan_bf16_s$SEED.log 2>&1
  rc=$?
  echo "seed $SEED rc=$rc $(tail -1 gpurun_out/r06e_scan_bf16_s$SEED.log | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 124 ]; then exit $rc; fi
done
