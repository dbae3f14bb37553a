#!/bin/bash
# r05w (lab knob since removed: profiles/r05w_attn_stagger_ab.txt): do the four attn_fwd_l2 workgroups of a CU run in lockstep?  Lab builds start blocks b + 256 k (the CU's
# k-th workgroup) k x S s_sleep units late (st16 / st32 / st64); tools/lab/attn_probe.py (the product kernel at
# large-v3 B = 32) and the bench's encoder pass, three alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base st16 st32 st64; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/lab/attn_probe.py 2>/dev/null) $(timeout -k 10 200 python tools/enc_pass.py --streams 2 --reps 3 2>/dev/null | tail -1)" >> gpurun_out/r05w_attn_ab.txt || exit 1
  done
done
cat gpurun_out/r05w_attn_ab.txt
