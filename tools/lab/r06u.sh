#!/bin/bash
# r06u: cross_attn_row_kernel with a fourth K / V buffer -- a 32 KB LDS slot for the even chunks' K (LDS-DMA), so
# the next chunk's K and V are in flight while a chunk is waited on (128 KB per pair instead of 96); plus r06t's
# level-by-level helper sums: bitwise vs HEAD (decode linears + every decode attention kernel), tests, kbench A/B,
# bench A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python tools/lab/declin_bitwise.py gpurun_out/r06u_new.npz > gpurun_out/r06u_bitwise.log 2>&1 &&
env KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so timeout -k 10 240 python tools/lab/declin_bitwise.py gpurun_out/r06u_old.npz >> gpurun_out/r06u_bitwise.log 2>&1 &&
python tools/lab/declin_bitwise.py --compare gpurun_out/r06u_new.npz gpurun_out/r06u_old.npz && rm -f gpurun_out/r06u_new.npz gpurun_out/r06u_old.npz &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "cross or xq or qkv or self_attn or beam or tokens_identical" > gpurun_out/r06u_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06u_pytest.log &&
for v in base lab base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 150 python tools/kbench.py --only xq_cross,cross_attn,qkv_self > gpurun_out/r06u_kb_$v.json 2> gpurun_out/r06u_kb.err && echo "$v $(tail -c 300 gpurun_out/r06u_kb_$v.json)" || { tail -5 gpurun_out/r06u_kb.err; exit 1; }
done &&
bash tools/lab/ab_lib.sh 2
