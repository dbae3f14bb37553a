#!/bin/bash
# r05u (ran on a lab knob since removed: profiles/r05u_lmh_even_ab.txt): LM head groups dealt evenly over all CUs (KW_LMH_EVEN=1: 256 workgroups of 6-7 column groups) vs runs of
# 7 (232 workgroups, 24 CUs idle): LM head tests, kbench (3 rounds), then bench.py both ways.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
KW_LMH_EVEN=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lm_head or dec_linear or greedy" > gpurun_out/r05u_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -2 gpurun_out/r05u_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for v in runs even; do
    case $v in runs) unset KW_LMH_EVEN ;; even) export KW_LMH_EVEN=1 ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only lm_head 2>/dev/null)" >> gpurun_out/r05u_lmh_ab.txt || exit 1
  done
done
cat gpurun_out/r05u_lmh_ab.txt
unset KW_LMH_EVEN
timeout -k 10 300 python bench.py > gpurun_out/r05u_bench_runs.json 2> gpurun_out/r05u_bench_runs.err || exit 1
KW_LMH_EVEN=1 timeout -k 10 300 python bench.py > gpurun_out/r05u_bench_even.json 2> gpurun_out/r05u_bench_even.err || exit 1
python -c "
import json
for f in ('gpurun_out/r05u_bench_runs.json','gpurun_out/r05u_bench_even.json'):
    d=json.load(open(f)); print(f, round(d['value'],1), d['decode_step_ms'], d['decode_kernel_us']['lm_head'])"
