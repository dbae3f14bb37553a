#!/bin/bash
# r05m: gemm256 main-loop issue order (lab builds: p5 = static priority for group 1, p6 = no s_setprio, p7 = group 0's
# A pieces interleaved with its fragment reads) -- tools/gemm_bench.py, three rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base p5 p6 p7; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null)" >> gpurun_out/r05m_gemm_ab.txt || exit 1
  done
done
cat gpurun_out/r05m_gemm_ab.txt
