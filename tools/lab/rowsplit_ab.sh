#!/bin/bash
# r04: the decode linears' row split (two 16-row chunks for grids of <= 128 column groups: o / xo) A/B through the lab
# build's KW_DECLIN_ROWSPLIT=0 switch (ctypes backend).
#   make -C kotoba-whisper_amd/csrc EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab OUT=../kwhisper/libkwhisper_lab.so \
#        TORCH_OUT=../kwhisper/libkwhisper_torch_lab.so
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export KWHISPER_LIB="$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so"
for rep in 1 2 3; do
  for on in 1 0; do
    echo -n "KW_DECLIN_ROWSPLIT=$on "
    KW_DECLIN_ROWSPLIT=$on timeout -k 10 120 python tools/kbench.py --backend ctypes --reps 40 --only o_resid,xq_ln,fc1_ln_gelu,o_plain 2>/dev/null || exit 1
  done
done
