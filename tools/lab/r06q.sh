#!/bin/bash
# r06q: the wave index read as a scalar (readfirstlane) in dec_linear / decproj / qkv_self / lm_head: wave-uniform
# branches become scalar branches, the k-range arithmetic scalar (VALU -8..-20 %); bitwise vs HEAD (declin_bitwise),
# kernel tests, kbench A/B of every decode-step kernel, decode-step A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LABENV="KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so"
timeout -k 10 180 python tools/lab/declin_bitwise.py gpurun_out/r06q_new.npz > gpurun_out/r06q_bitwise.log 2>&1 &&
env KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so timeout -k 10 180 python tools/lab/declin_bitwise.py gpurun_out/r06q_old.npz >> gpurun_out/r06q_bitwise.log 2>&1 &&
python tools/lab/declin_bitwise.py --compare gpurun_out/r06q_new.npz gpurun_out/r06q_old.npz && rm -f gpurun_out/r06q_new.npz gpurun_out/r06q_old.npz &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "dec_linear or qkv or xq or lm_greedy or lm_head or tokens_identical or fused" > gpurun_out/r06q_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06q_pytest.log &&
for v in base lab base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 150 python tools/kbench.py --only qkv_ln,o_resid,xq_ln,fc1_ln_gelu,fc2_resid,xq_cross,qkv_self > gpurun_out/r06q_kb_$v.json 2> gpurun_out/r06q_kb.err && echo "$v $(tail -c 600 gpurun_out/r06q_kb_$v.json)" || { tail -5 gpurun_out/r06q_kb.err; exit 1; }
done &&
bash tools/lab/ab_lib.sh 2
