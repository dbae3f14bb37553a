#!/bin/bash
# r06n: the rows kernel's (> 32 rows: prefill, beam rows) epilogue through store_block16 -- bitwise vs the previous
# library, kernel tests, config 5 (beam rows) A/B and decode A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LAB="KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so"
timeout -k 10 180 python tools/lab/declin_bitwise.py gpurun_out/r06n_new.npz > gpurun_out/r06n_bitwise.log 2>&1 &&
env KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so timeout -k 10 180 python tools/lab/declin_bitwise.py gpurun_out/r06n_old.npz >> gpurun_out/r06n_bitwise.log 2>&1 &&
python tools/lab/declin_bitwise.py --compare gpurun_out/r06n_new.npz gpurun_out/r06n_old.npz && rm -f gpurun_out/r06n_new.npz gpurun_out/r06n_old.npz &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "dec_linear or beam or tiny or prefill or lm_head" > gpurun_out/r06n_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06n_pytest.log &&
for v in base lab base lab; do
  if [ $v = lab ]; then export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; else unset KWHISPER_LIB KWHISPER_TORCH_LIB; fi
  timeout -k 10 200 python tools/bench_configs.py --config 5 --clips 64 > gpurun_out/r06n_c5_$v.json 2>/dev/null && echo "$v config5 $(python -c "import json;print(round(json.load(open('gpurun_out/r06n_c5_$v.json'))['value'],1))")"
done
