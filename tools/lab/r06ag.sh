#!/bin/bash
# r06ag: attn_fwd_l2 with block 1's score MFMAs beside block 0's exponentials (build_lab/il1: -DKW_ATTN_IL=1; il2: the
# interleave pinned by sched_group_barrier) vs the product: output hashes (bitwise) and time, interleaved rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base il1 il2; do
    if [ $v = base ]; then unset KWHISPER_LIB KWHISPER_TORCH_LIB; else export KWHISPER_LIB=$PWD/build_lab/$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/$v/libkwhisper_torch.so; fi
    timeout -k 10 120 python tools/lab/attn_lib_ab.py > gpurun_out/r06ag.json 2> gpurun_out/r06ag.err || { echo "FAIL $v"; tail -5 gpurun_out/r06ag.err; exit 1; }
    echo "$v $(cat gpurun_out/r06ag.json)"
  done
done
