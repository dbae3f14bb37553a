#!/bin/bash
# r05p: the bench's two-row-block encoder (tools/enc_pass.py --streams 2, large-v3 B = 32) with the gemm256 read-slot
# variants of r05n (p7 / p8 / p9 lab builds) against the product, three alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base p7 p8 p9; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 200 python tools/enc_pass.py --streams 2 --reps 5 2>/dev/null | tail -3 | tr '\n' ' ')" >> gpurun_out/r05p_enc_ab.txt || exit 1
  done
done
cat gpurun_out/r05p_enc_ab.txt
