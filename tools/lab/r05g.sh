#!/bin/bash
# r05g: LM head decomposition (lab builds: lmh1 = no epilogue stores, lmh2 = the weight stream alone).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in base lmh1 lmh2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only lm_head 2>/dev/null)" >> gpurun_out/r05g_ab.txt || exit 1
  done
done
cat gpurun_out/r05g_ab.txt
