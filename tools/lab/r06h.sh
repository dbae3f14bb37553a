#!/bin/bash
# r06h: decproj.h's reduction / publish spread over the two row halves (qkv_self, xq_cross) -- kernel tests, kbench
# of the fused blocks in both libraries, A/B of the decode step vs the previous library (build_lab/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "qkv_self or xq_cross or cross or self_attn or fused or handoff or tiny or greedy" > gpurun_out/r06h_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06h_pytest.log &&
for v in base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 120 python tools/kbench.py --only qkv_self,xq_cross --reps 40 > gpurun_out/r06h_kbench_$v.json 2>/dev/null && echo "$v $(tail -1 gpurun_out/r06h_kbench_$v.json | cut -c1-200)"
done
unset KWHISPER_LIB KWHISPER_TORCH_LIB
timeout -k 10 500 bash tools/lab/ab_lib.sh 2 > gpurun_out/r06h_ab.txt 2>&1; cat gpurun_out/r06h_ab.txt | cut -c1-60
