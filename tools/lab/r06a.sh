#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v -s --timeout 120 --timeout-method thread -k "lm_greedy or embed_mirror or steps_per_replay or stop_check or greedy_step or dec_linear_layernorm" > gpurun_out/r06a_pytest.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 python bench.py > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err && cat gpurun_out/r06a_bench.json
