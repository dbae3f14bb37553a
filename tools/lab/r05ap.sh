#!/bin/bash
# r05ap: the all-rows LM head on eight 16-column waves with four k-tile slices staged ahead (one workgroup per CU)
# instead of four waves with two ahead -- LM head / LayerNorm-linear / beam GPU tests, then its time vs rows and
# config 5 before (build_lmr0: the previous HEAD) and after.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py tests/test_gpu_workloads.py -m gpu -x -v --timeout 120 --timeout-method thread -k "layernorm or lm_head or beam or config5" > gpurun_out/r05ap_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/r05ap_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in tree lmr0; do
    case $v in tree) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/lab/lmr_probe.py 33 64 128 192 256 320 2>/dev/null)" >> gpurun_out/r05ap_lmr.txt || exit 1
  done
done
for v in tree lmr0; do
  case $v in tree) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
  echo "$v $(timeout -k 10 200 python tools/bench_configs.py --config 5 --clips 64 2>/dev/null | cut -c1-160)" >> gpurun_out/r05ap_config5.txt || exit 1
done
cat gpurun_out/r05ap_lmr.txt gpurun_out/r05ap_config5.txt
