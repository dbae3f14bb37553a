#!/bin/bash
# r06r: wave index as a scalar in the attention kernels and the LayerNorm row index (one row per wave); bench.py on
# the numpy-recipe model (the config-3 fixture's): full GPU suite, kbench xq_cross A/B, bench A/B (encoder + decode)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r06r_pytest_gpu.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06r_pytest_gpu.log &&
for v in base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 150 python tools/kbench.py --only xq_cross,cross_attn > gpurun_out/r06r_kb_$v.json 2> gpurun_out/r06r_kb.err && echo "$v $(tail -c 300 gpurun_out/r06r_kb_$v.json)" || { tail -5 gpurun_out/r06r_kb.err; exit 1; }
done &&
for r in 1 2; do
  for v in base lab; do
    if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r06r_bench_$v.json 2> gpurun_out/r06r_bench.err || { echo "FAIL $v"; tail -5 gpurun_out/r06r_bench.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r06r_bench_$v.json')); print('$v', round(d['value'],1), round(d['decode_step_ms'],3), round(d['encoder_mfma']['ms'],2), d['data'][-40:])"
  done
done
