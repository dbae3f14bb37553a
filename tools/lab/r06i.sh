#!/bin/bash
# r06i: fc2's K-split seam per (column group, row half) on two waves -- bitwise vs the previous library, kernel
# tests, chain stamps, decode-step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/lab/declin_bitwise.py gpurun_out/r06i_new.npz > gpurun_out/r06i_bitwise.log 2>&1 &&
KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so timeout -k 10 120 python tools/lab/declin_bitwise.py gpurun_out/r06i_old.npz >> gpurun_out/r06i_bitwise.log 2>&1 &&
python tools/lab/declin_bitwise.py --compare gpurun_out/r06i_new.npz gpurun_out/r06i_old.npz && rm -f gpurun_out/r06i_new.npz gpurun_out/r06i_old.npz &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "dec_linear or greedy or tiny or fused" > gpurun_out/r06i_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06i_pytest.log &&
timeout -k 10 120 ./tools/lab/chain_stamps.bin > gpurun_out/r06i_chain_stamps.txt 2>&1 && grep -E "^o|^fc|^qkv" gpurun_out/r06i_chain_stamps.txt | awk 'NR%3==1' | cut -c1-60 &&
timeout -k 10 500 bash tools/lab/ab_lib.sh 2 > gpurun_out/r06i_ab.txt 2>&1; cat gpurun_out/r06i_ab.txt | cut -c1-60
