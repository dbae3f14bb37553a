set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x12_pytest.log 2>&1; echo pytest rc $?; tail -2 gpurun_out/x12_pytest.log
timeout -k 10 100 python tools/kbench.py --only cross_attn,self_attn_t132,o_resid 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/x12_bench.json 2> gpurun_out/x12_bench.err; cat gpurun_out/x12_bench.json
