#!/bin/bash
# r06o: cross_attn_row_kernel's K / V pieces through buffer resources (one add per piece instead of a clamp and
# 64-bit address arithmetic) and the chunk-end check only on key group 7 (-15 % VALU, 165 -> 150 VGPRs):
# + fc2's split-major XCD deal (placement only);
# cross-attention and decode-linear tests (bitwise batch invariance vs the chunk-grid kernel), kbench A/B, decode step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "cross or xq or dec_linear" > gpurun_out/r06o_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06o_pytest.log &&
for v in base lab base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 120 python tools/kbench.py --only xq_cross,cross_attn,fc2_resid > gpurun_out/r06o_kb_$v.json 2> gpurun_out/r06o_kb.err && echo "$v $(tail -c 400 gpurun_out/r06o_kb_$v.json)" || { tail -5 gpurun_out/r06o_kb.err; exit 1; }
done &&
bash tools/lab/ab_lib.sh 2
