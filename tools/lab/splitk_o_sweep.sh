#!/bin/bash
# r04: K-split geometries for the decode step's residual linears (o / xo: N 1280 x K 1280; fc2: 1280 x 5120)
# through the KW_DECLIN_GEO="N,K,ncb,ktm,ks" override of a lab build (ctypes backend).
#   make -C kotoba-whisper_amd/csrc EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab OUT=../kwhisper/libkwhisper_lab.so \
#        TORCH_OUT=../kwhisper/libkwhisper_torch_lab.so
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export KWHISPER_LIB="$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so"
for rep in 1 2; do
  for cfg in default 1280,1280,1,5,2 1280,1280,1,5,4 1280,1280,1,10,2 1280,1280,1,10,4 \
             1280,5120,1,10,8 1280,5120,1,5,8 1280,5120,1,10,4 1280,5120,1,5,6; do
    if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=$cfg; fi
    echo -n "$cfg "
    timeout -k 10 120 python tools/kbench.py --backend ctypes --reps 40 --only o_resid,fc2_resid 2>/dev/null || exit 1
  done
done
