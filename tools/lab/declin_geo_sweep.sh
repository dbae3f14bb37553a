#!/bin/bash
# Decode-linear geometry sweep (ks == 1 shapes) through the KW_DECLIN_GEO="N,K,ncb,ktm,ks" lab override.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# the override is compiled into lab builds only:
#   make -C kotoba-whisper_amd/csrc EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab OUT=../kwhisper/libkwhisper_lab.so
export KWHISPER_LIB="${KWHISPER_LIB:-$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so}"
for rep in 1 2; do
  for cfg in default 1280,1280,1,5,1 1280,1280,2,5,1 5120,1280,1,5,1 5120,1280,1,10,1 5120,1280,2,5,1 3840,1280,1,10,1 3840,1280,2,5,1 3840,1280,2,10,1; do
    if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=$cfg; fi
    echo -n "$cfg "
    timeout -k 10 120 python tools/kbench.py --reps 40 --only qkv_ln,o_resid,xq_ln,fc1_ln_gelu 2>/dev/null || exit 1
  done
done
