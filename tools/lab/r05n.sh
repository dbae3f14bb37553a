#!/bin/bash
# r05n: gemm256 read-slot issue order (lab builds: p7 = group 0 interleaves its A pieces with its reads, p8 = p7 + group 1
# reads its W rows first, then interleaves its W pieces with the A reads; p9 = p8 with each piece after its reads)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base p7 p8 p9; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null)" >> gpurun_out/r05n_gemm_ab.txt || exit 1
  done
done
cat gpurun_out/r05n_gemm_ab.txt
