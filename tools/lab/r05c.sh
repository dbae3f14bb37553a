#!/bin/bash
# r05c: the engine's own seek trajectory on the config-4 HIP log-mel fixture (bf16 / fp32), the whole GPU test suite,
# the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/dump_trajectory.py --out gpurun_out/c4_traj.npz > gpurun_out/r05c_traj.log 2>&1 || { tail -20 gpurun_out/r05c_traj.log; exit 1; }
cat gpurun_out/r05c_traj.log | grep -v amdgpu.ids
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -s --maxfail 6 --timeout 300 --timeout-method thread > gpurun_out/r05c_pytest_gpu.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -15 gpurun_out/r05c_pytest_gpu.log; [ $rc -ge 124 ] && exit 1
timeout -k 10 300 python bench.py > gpurun_out/r05c_bench.json 2> gpurun_out/r05c_bench.err && cat gpurun_out/r05c_bench.json
