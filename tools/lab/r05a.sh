#!/bin/bash
# r05a (lab, not product): HIP log-mel dump for the config-4 fixture, LM head / decode-linear tests, the large-v3 fp32
# logits and long-form per-pass checks, cold lanes; then the LM head A/B: product (3 buffers) vs build_lab (2) vs
# build_lab2 (round-4 kernel), kbench and bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
crash() { [ "$1" -ge 124 ]; }
timeout -k 10 240 python -u tools/dump_hipmel.py --out gpurun_out/c4_hipmel_features.npz > gpurun_out/r05a_dump.log 2>&1 || exit 1
echo DUMP_OK
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dec_linear or mlp" > gpurun_out/r05a_kern.log 2>&1
rc=$?; echo "KERN rc=$rc"; crash $rc && exit 1
timeout -k 10 700 python -u -m pytest -m gpu -x -v -s --timeout 300 --timeout-method thread \
  "tests/test_gpu_workloads.py::test_config3_fp32_generate_b32_bitexact" \
  "tests/test_gpu_workloads.py::test_large_v3_longform_multipass[large_v3_longform_fp32]" \
  "tests/test_gpu_workloads.py::test_lanes_cold_capture_multipass" \
  "tests/test_gpu_workloads.py::test_config3_bf16_generate_b32" > gpurun_out/r05a_work.log 2>&1
rc=$?; echo "WORK rc=$rc"; crash $rc && exit 1
for r in 1 2; do
  for v in base lab lab2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only lm_head 2>/dev/null)" >> gpurun_out/r05a_lmh_ab.txt || exit 1
  done
done
for r in 1 2; do
  for v in base lab2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    echo "$v $(timeout -k 10 120 python tools/kbench.py --reps 40 --only mlp,fc1_ln_gelu,fc2_resid 2>/dev/null)" >> gpurun_out/r05a_lmh_ab.txt || exit 1
  done
done
for r in 1 2; do
  for v in base lab2; do
    case $v in base) unset KWHISPER_LIB KWHISPER_TORCH_LIB ;; *) export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so ;; esac
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05a_ab.json 2> gpurun_out/r05a_ab.err || { echo "FAIL $v"; tail -5 gpurun_out/r05a_ab.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r05a_ab.json')); print('$v', round(d['value'],1), round(d['decode_step_ms'],3), d['decode_kernel_us'])" >> gpurun_out/r05a_lmh_ab.txt
  done
done
cat gpurun_out/r05a_lmh_ab.txt
