#!/bin/bash
# r05ac: the log-mel's mel projection over each filter's nonzero bins only -- the fixture log-mel bitwise and the
# oracle tolerance tests, then kw_log_mel's time (large-v3, B = 32, 30 s) before (build_mel0: the previous HEAD) and after.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_workloads.py -m gpu -x -v --timeout 120 --timeout-method thread -k "log_mel or hipmel_fixture" > gpurun_out/r05ac_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/r05ac_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for v in tree mel0; do
    case $v in tree) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/lab/mel_probe.py 2>/dev/null)" >> gpurun_out/r05ac_mel.txt || exit 1
  done
done
cat gpurun_out/r05ac_mel.txt
