#!/bin/bash
# r05l: encoder GEMM epilogue decomposition (lab builds: ga1 = GELU on the accumulators, ga2 = the same with packed f32;
# results bitwise the product's) -- tools/gemm_bench.py, three rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base ga1 ga2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null)" >> gpurun_out/r05l_gemm_ab.txt || exit 1
  done
done
cat gpurun_out/r05l_gemm_ab.txt
