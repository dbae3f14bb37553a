#!/bin/bash
# r06d: config-4 multi-pass scan on other numpy-recipe seeds (fp32 engine, bit-exact with transformers fp32)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for SEED in ${SEEDS:-1}; do
  timeout -k 10 ${PER:-560} python -u tools/find_multipass.py --weights numpy --seed $SEED --dtype float32 --n-clips 1768 \
    --stop-after 2 --out gpurun_out/r06d_multipass_s$SEED.json --features-out gpurun_out/r06d_multipass_s${SEED}_features.npz \
    > gpurun_out/r06d_scan_s$SEED.log 2>&1
  rc=$?
  tail -2 gpurun_out/r06d_scan_s$SEED.log
  if [ $rc -ne 0 ] && [ $rc -ne 124 ]; then exit $rc; fi
done
