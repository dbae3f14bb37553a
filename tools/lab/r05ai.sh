#!/bin/bash
# r05ai: as r05ah, the LayerNorm statistics computed by each epilogue job's wave for its row half (no second barrier)
# instead of wave 0 alone -- the rows-kernel bitwise tests, then the device time per call at M = 128 / 320
# before (build_rows0: the previous HEAD) and after.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "dec_linear or lm_head" > gpurun_out/r05ai_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/r05ai_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for v in tree rows0; do
    case $v in tree) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/lab/rows_probe.py 2>/dev/null)" >> gpurun_out/r05ai_rows.txt || exit 1
  done
done
cat gpurun_out/r05ai_rows.txt
