set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "self_attn or cross_attn" > gpurun_out/x13_pytest.log 2>&1; echo pytest rc $?; tail -1 gpurun_out/x13_pytest.log
timeout -k 10 100 python tools/kbench.py --only self_attn_t132 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/x13_bench.json 2> gpurun_out/x13_bench.err; python -c "import json;d=json.load(open('gpurun_out/x13_bench.json'));print(d['value'],d['decode_step_ms'],d['decode_kernel_us'])"
