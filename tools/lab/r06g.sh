#!/bin/bash
# r06g: kw_dec_linear epilogue spread over the (column block, row half) jobs -- kernel tests, chain stamps, A/B vs
# the previous library (build_lab/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "dec_linear or lm_greedy or greedy or embed or tiny or steps_per_replay or stop_check or fused" > gpurun_out/r06g_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06g_pytest.log &&
timeout -k 10 120 ./tools/lab/chain_stamps.bin > gpurun_out/r06g_chain_stamps.txt 2>&1 && grep -E "^o|^fc|^qkv" gpurun_out/r06g_chain_stamps.txt | awk 'NR%3==1' | cut -c1-60 &&
timeout -k 10 500 bash tools/lab/ab_lib.sh 2 > gpurun_out/r06g_ab.txt 2>&1; cat gpurun_out/r06g_ab.txt | cut -c1-60
