#!/bin/bash
# LM head A/B: in-tree library vs the r02j build in build_lab/ (kbench lm_head, then bench.py via ab_lib.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lm_head or logits or large or beam or greedy" > gpurun_out/l_tests.log 2>&1 && echo TESTS_OK || { tail -30 gpurun_out/l_tests.log; exit 1; }
for r in 1 2; do
  for v in base lab; do
    if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only lm_head 2>/dev/null)" >> gpurun_out/l_ab.txt || exit 1
  done
done
unset KWHISPER_LIB KWHISPER_TORCH_LIB
timeout -k 10 500 bash tools/lab/ab_lib.sh 2 >> gpurun_out/l_ab.txt 2>&1
