#!/bin/bash
# fc2 (N 1280, K 5120) geometry sweep through the KW_DECLIN_GEO="N,K,ncb,ktm,ks" lab override: two column
# blocks per workgroup halve the activation re-reads (80 column groups x 327 KB of x at ncb 1), at the cost
# of fewer workgroups.  Lab build (override compiled in) in build_lab/:
#   make -C kotoba-whisper_amd/csrc EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab \
#        OUT=../../build_lab/libkwhisper.so TORCH_OUT=../../build_lab/libkwhisper_torch.so
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so
for rep in 1 2; do
  for cfg in default 1280,5120,2,10,6 1280,5120,2,10,3 1280,5120,2,10,2 1280,5120,2,5,8 1280,5120,2,5,4 1280,5120,1,5,8 1280,5120,1,10,4; do
    if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=$cfg; fi
    echo -n "$cfg "
    timeout -k 10 120 python tools/kbench.py --reps 40 --only fc2_resid 2>/dev/null || exit 1
  done
done
