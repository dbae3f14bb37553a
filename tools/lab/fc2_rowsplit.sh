#!/bin/bash
# r04: fc2 (N 1280 x K 5120, K-split) with and without the row split (KW_DECLIN_ROWSPLIT=2 lets the K-split grids
# run two 16-row chunks too) over K-split geometries (KW_DECLIN_GEO="N,K,ncb,ktm,ks"; lab build, ctypes backend).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# lab library: bash tools/lab/mlp_lab_build.sh tools/lab/fc2_rowsplit.diff
export KWHISPER_LIB="$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so"
for rep in 1 2; do
  for cfg in default 1280,5120,1,10,3 1280,5120,1,10,4 1280,5120,1,5,4 1280,5120,1,5,8; do
    for mode in 1 2; do
      if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=$cfg; fi
      echo -n "$cfg rowsplit=$mode "
      KW_DECLIN_ROWSPLIT=$mode timeout -k 10 120 python tools/kbench.py --backend ctypes --reps 40 --only fc2_resid 2>/dev/null || exit 1
    done
  done
done
