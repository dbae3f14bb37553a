#!/bin/bash
# r05b (lab, not product): decode-linear / LM head / fused-MLP kernel tests; the fused MLP decomposed (build_m1: fc2
# without waits, build_m2: the fc1 role alone, build_m3: the fc2 role alone, no waits; results wrong, timings real);
# FETCH of the row-split o-projection with default-policy weight loads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dec_linear or mlp" > gpurun_out/r05b_kern.log 2>&1
rc=$?; echo "KERN rc=$rc"; [ $rc -ge 124 ] && exit 1
for r in 1 2; do
  for v in base m1 m2 m3; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only mlp,fc1_ln_gelu,fc2_resid,o_resid,lm_head 2>/dev/null)" >> gpurun_out/r05b_ab.txt || exit 1
  done
done
unset KWHISPER_LIB KWHISPER_TORCH_LIB
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d /tmp/r05b_pmc -o run -- python3 tools/kbench.py --eager --reps 2 --only o_resid,lm_head,fc2_resid,fc1_ln_gelu > gpurun_out/r05b_pmc.log 2>&1 &&
python3 tools/rocpd_summary.py --pmc /tmp/r05b_pmc/run_results.db gpurun_out/r05b_pmc_fetch.csv
cat gpurun_out/r05b_ab.txt; cat gpurun_out/r05b_pmc_fetch.csv
