#!/bin/bash
# Lab A/B (not product): bench.py decode step with the in-tree library vs a lab build in build_lab/
# (KWHISPER_LIB / KWHISPER_TORCH_LIB), interleaved.   bash tools/lab/ab_lib.sh [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for r in $(seq ${1:-2}); do
  for v in base lab; do
    if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_lib.json 2> gpurun_out/ab_lib.err || { echo "FAIL $v"; tail -5 gpurun_out/ab_lib.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_lib.json')); print('$v', round(d['value'],1), round(d['decode_step_ms'],3), d['decode_kernel_us'])"
  done
done
