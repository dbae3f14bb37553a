#!/bin/bash
# fc2 (N 1280, K 5120) split-K geometry sweep through the KW_DECLIN_GEO lab override (N,K,ncb,ktm,ks) (tools/kbench.py).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# the override is compiled into lab builds only:
#   make -C kotoba-whisper_amd/csrc EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab OUT=../kwhisper/libkwhisper_lab.so
export KWHISPER_LIB="${KWHISPER_LIB:-$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so}"
mkdir -p gpurun_out
for cfg in default 5,8 10,4 5,4 10,5 10,6 10,2 default; do
  if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=1280,5120,1,$cfg; fi
  echo -n "$cfg "
  timeout -k 10 120 python tools/kbench.py --reps 40 --only fc2_resid,o_resid || exit 1
done
