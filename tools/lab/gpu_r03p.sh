set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/kbench.py --only xq_cross,cross_attn,qkv_self,self_attn --reps 20 > gpurun_out/r03p_kbench.json 2>&1 && cat gpurun_out/r03p_kbench.json &&
KW_CROSS_ROW=0 timeout -k 10 300 python -u tools/kbench.py --only xq_cross,cross_attn --reps 20 > gpurun_out/r03p_kbench_row0.json 2>&1 && cat gpurun_out/r03p_kbench_row0.json &&
bash tools/pmc_only.sh r03p &&
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03p_bench.json 2> gpurun_out/r03p_bench.err && cat gpurun_out/r03p_bench.json
