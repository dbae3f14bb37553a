#!/bin/bash
# Lab (not product): tools/lab/chain_lab.py over decode-linear geometries (lab build in build_lab/ with
# KW_LAB_OVERRIDES: KW_DECLIN_GEO="N,K,ncb,ktm,ks;...").   bash tools/lab/chain_sweep.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so
for geo in "" "1280,5120,1,5,6" "1280,5120,1,5,4" "5120,1280,1,5,1;1280,5120,1,5,4" "5120,1280,1,5,1;1280,5120,1,5,6"; do
  echo "== KW_DECLIN_GEO=$geo"
  KW_DECLIN_GEO="$geo" timeout -k 10 120 python -u tools/lab/chain_lab.py --iters 10 2>/dev/null | tail -1 || exit 1
done
