#!/bin/bash
# r05d: the LM head fix on the tiny shapes (kernel + generate tests), the RCCL test; the batch-size probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py tests/test_gpu_dist.py -m gpu -q --maxfail 4 --timeout 300 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -8 gpurun_out/r05d_tests.log; [ $rc -ge 124 ] && exit 1
timeout -k 10 300 python -u tools/lab/batch_probe.py --dtype bfloat16 > gpurun_out/r05d_probe_bf16.json 2> gpurun_out/r05d_probe.err && cat gpurun_out/r05d_probe_bf16.json
timeout -k 10 300 python -u tools/lab/batch_probe.py --dtype float32 > gpurun_out/r05d_probe_fp32.json 2>> gpurun_out/r05d_probe.err && cat gpurun_out/r05d_probe_fp32.json
