#!/bin/bash
# rocprofv3 passes behind profiles/ (run on the GPU box): kernel-trace stats of the bench, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes over the decode kernels (tools/kbench.py, eager).
#   bash tools/profile.sh r01   -> gpurun_out/<tag>_bench_prof, <tag>_pmc_fetch, <tag>_pmc_write
set -e
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_bench_prof -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/${TAG}_bench_prof.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_fetch -o run -- python3 tools/kbench.py --eager --reps 2 --only cross_attn,self_attn,o_resid,fc1_ln_gelu,fc2_resid,qkv_ln,xq_ln,lm_head > gpurun_out/${TAG}_pmc_fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/${TAG}_pmc_write -o run -- python3 tools/kbench.py --eager --reps 2 --only cross_attn,self_attn,o_resid,fc1_ln_gelu,fc2_resid,qkv_ln,xq_ln,lm_head > gpurun_out/${TAG}_pmc_write.log 2>&1
# the kernel sources these counters measured (bench.py reports roofline.traffic only for the same sources)
python3 -c "import bench, json; print(json.dumps({'kernel_source_sha256': bench.kernel_source_hash()}))" > gpurun_out/${TAG}_pmc_fetch.meta.json
tail -1 gpurun_out/${TAG}_bench_prof.log
