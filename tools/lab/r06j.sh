#!/bin/bash
# r06j: config 4's short-clip multi-pass fixture (numpy seed 6) and the other config-4 tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_workloads.py -x -v -s --timeout 300 --timeout-method thread -k "config4" > gpurun_out/r06j_pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|config4|passed|failed" gpurun_out/r06j_pytest.log | tail -20; exit $rc
