set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/overlap2_lab.py > gpurun_out/r03b_overlap2.log 2>&1 && echo LAB_OK &&
bash tools/profile.sh r03b && echo PROF_OK &&
timeout -k 10 500 python -u tools/cpu_ref_rate.py --batch 32 > gpurun_out/r03_cpu_baseline_b32.json 2> gpurun_out/r03_cpu_baseline_b32.err && cat gpurun_out/r03_cpu_baseline_b32.json
