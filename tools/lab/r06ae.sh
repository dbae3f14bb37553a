#!/bin/bash
# r06ae: gemm256 with four read / MFMA phases per K-tile (-DKW_GEMM_PH8=1, build_lab/) vs the product's two slots:
# output hashes (must be bitwise equal: same MFMA order per accumulator) and times per encoder GEMM, interleaved;
# then the tile timeline (tools/lab/gemm_lab.hip) of both builds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2; do
  for g in fc1 qkv o fc2; do
    for v in base lab; do
      if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
      timeout -k 10 120 python tools/lab/gemm_ab.py $g > gpurun_out/r06ae_ab.json 2> gpurun_out/r06ae_ab.err || { echo "FAIL $v $g"; tail -5 gpurun_out/r06ae_ab.err; exit 1; }
      echo "$v $(cat gpurun_out/r06ae_ab.json)"
    done
  done
done
for m in "48000 1280 1280 0" "48000 1280 1280 2" "48000 5120 1280 1" "48000 1280 5120 2"; do
  timeout -k 10 30 ./tools/lab/gemm_lab.bin $m | head -2 && timeout -k 10 30 ./tools/lab/gemm_lab_ph8.bin $m | head -2 || exit 1
done
