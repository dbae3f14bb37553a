#!/bin/bash
# r05x (ran on a build since reverted: profiles/r05x_gelu_table_ab.txt): fc1 / conv1 GELU by LDS table (that build, KW_GEMM_GELU_TAB=1: the bf16-rounded x + bias looked up in a
# 10 KB table of the reference's bf16 GELU) vs per-element GELU of the f32 value (build_gt0: -DKW_GEMM_GELU_TAB=0);
# GEMM tests on the table build, then tools/gemm_bench.py and the bench's encoder pass, three alternating rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/r05x_tests.log 2>&1
rc=$?; echo "TESTS rc=$rc"; tail -3 gpurun_out/r05x_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for v in gt0 tab; do
    case $v in tab) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null) $(timeout -k 10 200 python tools/enc_pass.py --streams 2 --reps 3 2>/dev/null | tail -1)" >> gpurun_out/r05x_ab.txt || exit 1
  done
done
python - <<'PY'
import json
for line in open('gpurun_out/r05x_ab.txt'):
    v, rest = line.split(' ', 1)
    js, enc = rest.split('} encoder', 1)
    d = json.loads(js + '}')
    print(v, 'fc1', d['fc1_gelu']['us'], 'qkv', d['qkv_headsplit']['us'], 'fc2', d['fc2_store_bf16']['us'], 'encoder' + enc.strip())
PY
