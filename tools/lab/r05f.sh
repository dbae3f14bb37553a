#!/bin/bash
# r05f: the fused self block's projection by 16-row chunks (product) vs the round-4 block (build_lab2): kernel tests
# of the fused blocks, kbench qkv_self, bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -m gpu -q --maxfail 3 --timeout 200 --timeout-method thread -k "qkv_self or fused or handoff or greedy or large" > gpurun_out/r05f_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -5 gpurun_out/r05f_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in base lab2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only qkv_self --self-t 68,132 2>/dev/null)" >> gpurun_out/r05f_ab.txt || exit 1
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05f_ab.json 2> gpurun_out/r05f_ab.err || { echo "FAIL $v"; tail -5 gpurun_out/r05f_ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05f_ab.json')); print('$v', round(d['value'],1), round(d['decode_step_ms'],3), d['decode_kernel_us'])" >> gpurun_out/r05f_ab.txt
  done
done
for r in 1 2; do
  for v in base lmh1 lmh2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only lm_head 2>/dev/null)" >> gpurun_out/r05f_ab.txt || exit 1
  done
done
cat gpurun_out/r05f_ab.txt
