#!/bin/bash
# (ran against tools/lab/oxq_cross.diff applied; reverted -- profiles/r05z_oxq_cross_ab.txt)
# r05z: kw_dec_oxq_cross (the self block's out-projection in the cross block's launch) -- its parity tests, the
# cross-attention and decode tests, then bench.py with it (default) and without it (KW_OXQ=0), twice each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
crash() { [ "$1" -ge 124 ]; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "oxq or xq_cross or cross_attn_batch" > gpurun_out/r05z_kern.log 2>&1
rc=$?; echo "KERN rc=$rc"; tail -3 gpurun_out/r05z_kern.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py tests/test_gpu_generate.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config3 or greedy or b32 or status or fault" > gpurun_out/r05z_work.log 2>&1
rc=$?; echo "WORK rc=$rc"; tail -3 gpurun_out/r05z_work.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/r05z_bench_oxq$r.json 2> gpurun_out/r05z_bench_oxq$r.err || exit 1
  KW_OXQ=0 timeout -k 10 300 python bench.py > gpurun_out/r05z_bench_two$r.json 2> gpurun_out/r05z_bench_two$r.err || exit 1
done
python -c "
import json
for r in (1, 2):
    for v in ('oxq', 'two'):
        d = json.load(open(f'gpurun_out/r05z_bench_{v}{r}.json'))
        print(v, r, round(d['value'], 1), round(d['decode_step_ms'], 4), d['roofline']['avg_launch_us'])"
