#!/bin/bash
# r06y: the fused blocks' projection (decproj.h) with its fault word kept opaque (read as a uniform scalar up front it
# put a vmcnt(0) in front of every weight load) and its ten weight loads issued back to back from addresses formed
# first (a branch / address arithmetic among them drew more waits in qkv_self); direct activation fragments as
# before (r06x's LDS staging was slower): stamps, bitwise vs HEAD, tests, kbench A/B, bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 100 tools/lab/qkv_stamps.bin > gpurun_out/r06y_qkv_stamps.txt 2>&1 && cat gpurun_out/r06y_qkv_stamps.txt &&
timeout -k 10 240 python tools/lab/declin_bitwise.py gpurun_out/r06y_new.npz > gpurun_out/r06y_bitwise.log 2>&1 &&
env KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so timeout -k 10 240 python tools/lab/declin_bitwise.py gpurun_out/r06y_old.npz >> gpurun_out/r06y_bitwise.log 2>&1 &&
python tools/lab/declin_bitwise.py --compare gpurun_out/r06y_new.npz gpurun_out/r06y_old.npz && rm -f gpurun_out/r06y_new.npz gpurun_out/r06y_old.npz &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "cross or xq or qkv or self_attn or tokens_identical or handoff or fused" > gpurun_out/r06y_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06y_pytest.log &&
for v in base lab base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 150 python tools/kbench.py --only xq_cross,qkv_self > gpurun_out/r06y_kb_$v.json 2> gpurun_out/r06y_kb.err && echo "$v $(tail -c 300 gpurun_out/r06y_kb_$v.json)" || { tail -5 gpurun_out/r06y_kb.err; exit 1; }
done &&
bash tools/lab/ab_lib.sh 2
