#!/bin/bash
# r05s (ran on the split-pair build, since reverted: profiles/r05s_cross_split_ab.txt): split pairs in cross_attn_row_kernel -- parity (batch-invariance / split-pair tests, the greedy decode
# parity) and the A/B against the unsplit grid (KW_CROSS_SPLIT=0): tools/kbench.py xq_cross / cross_attn and the
# batch-size probe, then bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
crash() { [ "$1" -ge 124 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cross_attn" > gpurun_out/r05s_kern.log 2>&1
rc=$?; echo "KERN rc=$rc"; tail -3 gpurun_out/r05s_kern.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in split nosplit; do
    case $v in split) unset KW_CROSS_SPLIT ;; nosplit) export KW_CROSS_SPLIT=0 ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only xq_cross,cross_attn 2>/dev/null)" >> gpurun_out/r05s_ab.txt || exit 1
  done
done
unset KW_CROSS_SPLIT
timeout -k 10 300 python tools/lab/crossb_probe.py 13,16,20,25,26,32,35,38 > gpurun_out/r05s_crossb.txt 2>&1 || exit 1
cat gpurun_out/r05s_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_generate.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config3 or greedy or b32" > gpurun_out/r05s_work.log 2>&1
rc=$?; echo "WORK rc=$rc"; tail -3 gpurun_out/r05s_work.log; crash $rc && exit 1
timeout -k 10 300 python bench.py > gpurun_out/r05s_bench.json 2> gpurun_out/r05s_bench.err || exit 1
KW_CROSS_SPLIT=0 timeout -k 10 300 python bench.py > gpurun_out/r05s_bench_nosplit.json 2> gpurun_out/r05s_bench_nosplit.err || exit 1
python -c "
import json
for f in ('gpurun_out/r05s_bench.json','gpurun_out/r05s_bench_nosplit.json'):
    d=json.load(open(f)); print(f, round(d['value'],1), d['decode_step_ms'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
