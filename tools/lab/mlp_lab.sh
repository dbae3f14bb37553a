#!/bin/bash
# r04: where the fused MLP's (kw_dec_mlp) time goes: the lab build's KW_MLP_LAB skips fc2's fragment loads (1), its
# flag polls (2) or both (3) -- results are wrong, timings tell what each step costs -- beside the two launches.
#   make -C kotoba-whisper_amd/csrc EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab OUT=../kwhisper/libkwhisper_lab.so \
#        TORCH_OUT=../kwhisper/libkwhisper_torch_lab.so
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export KWHISPER_LIB="$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so"
for rep in 1 2; do
  for mode in 0 1 2 3; do
    echo -n "KW_MLP_LAB=$mode "
    KW_MLP_LAB=$mode timeout -k 10 120 python tools/kbench.py --backend ctypes --reps 40 --only fc1_ln_gelu,fc2_resid,mlp 2>/dev/null || exit 1
  done
done
