#!/bin/bash
# r05y (builds since reverted: profiles/r05y_epilogue_pipe_ab.txt): gemm256's bf16 epilogue software-pipelined (build ep1, -DKW_GEMM_EPI_PIPE=1: row piece s staged while piece
# s - 1 is finished and stored) vs the same sources without it (the tree: the epilogue's finishing code as a lambda)
# vs the committed r05v sources (build head).  GEMM tests on ep1, then gemm_bench + the encoder pass, 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
KWHISPER_LIB=$PWD/build_ep1/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_ep1/libkwhisper_torch.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r05y_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/r05y_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for v in head tree ep1; do
    case $v in tree) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null) $(timeout -k 10 200 python tools/enc_pass.py --streams 2 --reps 3 2>/dev/null | tail -1)" >> gpurun_out/r05y_ab.txt || exit 1
  done
done
python - <<'PY'
import json
for line in open('gpurun_out/r05y_ab.txt'):
    v, rest = line.split(' ', 1)
    js, enc = rest.split('} encoder', 1)
    d = json.loads(js + '}')
    print(v, 'qkv', d['qkv_headsplit']['us'], 'o', d['o_store_bf16']['us'], 'fc1', d['fc1_gelu']['us'], 'fc2', d['fc2_store_bf16']['us'], 'xkv', d['cross_kv_headsplit']['us'], 'encoder' + enc.strip())
PY
