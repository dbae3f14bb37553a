#!/bin/bash
# r05k: encoder GEMM epilogue decomposition (lab builds: g1 = fc1 without GELU, g2 = no bf16 epilogue stores;
# results wrong, timings real) -- tools/gemm_bench.py, three rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base g1 g2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null)" >> gpurun_out/r05k_gemm_ab.txt || exit 1
  done
done
cat gpurun_out/r05k_gemm_ab.txt
