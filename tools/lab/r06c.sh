#!/bin/bash
# r06c: the full GPU suite on the fused-tail tree, then the tail A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r06c_pytest_gpu.log 2>&1 && echo TESTS_OK && tail -3 gpurun_out/r06c_pytest_gpu.log &&
timeout -k 10 300 python tools/lab/tail_ab.py --rounds 3 > gpurun_out/r06c_tail_ab.txt 2>&1 && tail -1 gpurun_out/r06c_tail_ab.txt
