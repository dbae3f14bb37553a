#!/bin/bash
# r04: fc2 (N 1280 x K 5120) K-split counts 3 / 6 at 10 and 5 k-tiles per wave (ks 2 needs a 161-KB LDS image) (KW_DECLIN_GEO override of the lab
# build, ctypes backend; r04q found ks 3 x ktm 10 0.25 us under the default ks 6 x ktm 5).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export KWHISPER_LIB="$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so"
for rep in 1 2 3; do
  for cfg in default 1280,5120,1,10,3 1280,5120,1,10,6 1280,5120,1,5,6; do
    if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=$cfg; fi
    echo -n "$cfg "
    timeout -k 10 120 python tools/kbench.py --backend ctypes --reps 60 --only fc2_resid 2>/dev/null || exit 1
  done
done
