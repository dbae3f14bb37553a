set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sa_tests.log 2>&1 && echo TESTS_OK &&
timeout -k 10 120 python tools/kbench.py --reps 40 --only self_attn --self-t 4,32,68,100,132,300 > gpurun_out/sa_new.json 2>/dev/null &&
KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so timeout -k 10 120 python tools/kbench.py --reps 40 --only self_attn --self-t 4,32,68,100,132,300 > gpurun_out/sa_old.json 2>/dev/null &&
timeout -k 10 500 bash tools/lab/ab_lib.sh 2 > gpurun_out/sa_ab.txt 2>&1
