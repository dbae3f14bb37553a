#!/bin/bash
# Cross-attention chunking A/B: in-tree (256-key chunks, K by LDS-DMA) vs build_ng4d2 (128-key chunks, K and V
# by LDS-DMA, 32 KB LDS) vs build_ng4d1 (128-key chunks, K by LDS-DMA).  Kernel tests per variant, kbench, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
use() { if [ "$1" = base ]; then unset KWHISPER_LIB KWHISPER_TORCH_LIB; else export KWHISPER_LIB=$PWD/build_$1/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$1/libkwhisper_torch.so; fi; }
for v in ng4d2 ng4d1; do
  use $v
  timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "cross and not multirow" > gpurun_out/x_tests_$v.log 2>&1 && echo "TESTS_OK $v" || { echo "TESTS_FAIL $v"; tail -20 gpurun_out/x_tests_$v.log; exit 1; }
done
for r in 1 2; do
  for v in base ng4d2 ng4d1; do
    use $v
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only cross_attn 2>/dev/null)" || exit 1
  done
done
for r in 1 2; do
  for v in base ng4d2; do
    use $v
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/x_b.json 2> gpurun_out/x_b.err || { echo "BENCH_FAIL $v"; tail -5 gpurun_out/x_b.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/x_b.json')); print('$v', round(d['value'],1), round(d['decode_step_ms'],3), d['roofline']['avg_launch_us'])"
  done
done
