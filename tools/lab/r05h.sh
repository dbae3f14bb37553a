#!/bin/bash
# r05h: LM head with the run's logits staged in LDS and written back as row spans (product) vs per-group tile stores
# (build_lab2): decode-linear kernel tests, tiny generate tests, kbench, bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -m gpu -q --maxfail 3 --timeout 200 --timeout-method thread -k "dec_linear or tiny or large or greedy" > gpurun_out/r05h_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -5 gpurun_out/r05h_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in base lab2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only lm_head 2>/dev/null)" >> gpurun_out/r05h_ab.txt || exit 1
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05h_ab.json 2> gpurun_out/r05h_ab.err || { echo "FAIL $v"; tail -5 gpurun_out/r05h_ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05h_ab.json')); print('$v', round(d['value'],1), round(d['decode_step_ms'],3), d['decode_kernel_us'])" >> gpurun_out/r05h_ab.txt
  done
done
cat gpurun_out/r05h_ab.txt
