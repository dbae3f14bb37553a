#!/bin/bash
# r06p: cross_attn_row_kernel's fold on scalars (m_w, l_w read by readfirstlane: the fold mode a scalar branch instead
# of eight exec-masked ones per chunk; 127 -> 3 s_and_saveexec, VALU 3008 -> 2896): cross tests, kbench A/B vs HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "cross or xq" > gpurun_out/r06p_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06p_pytest.log &&
for v in base lab base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 120 python tools/kbench.py --only xq_cross,cross_attn > gpurun_out/r06p_kb_$v.json 2> gpurun_out/r06p_kb.err && echo "$v $(tail -c 300 gpurun_out/r06p_kb_$v.json)" || { tail -5 gpurun_out/r06p_kb.err; exit 1; }
done
