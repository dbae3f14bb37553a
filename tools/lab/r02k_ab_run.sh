#!/bin/bash
# r02k A/B on the GPU box: GPU tests on the in-tree library, then bench.py and config 5 with the in-tree
# library (base) vs the r02j build in build_lab/ (lab), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k_tests.log 2>&1 && echo TESTS_OK || { tail -30 gpurun_out/k_tests.log; exit 1; }
timeout -k 10 500 bash tools/lab/ab_lib.sh 2 > gpurun_out/k_ab.txt 2>&1 || exit 1
for v in base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 200 python tools/bench_configs.py --config 5 --clips 64 > gpurun_out/k_c5_$v.json 2> gpurun_out/k_c5_$v.err || exit 1
  echo "$v $(python -c "import json; print(round(json.load(open('gpurun_out/k_c5_$v.json'))['value'],1))")" >> gpurun_out/k_ab.txt
done
