# r03av lab, part 2: the sampler kernel's traced duration, in-tree (base) vs build_lab (one arrival count)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base lab; do
  if [ $v = base ]; then unset KWHISPER_LIB KWHISPER_TORCH_LIB; else export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r03av_$v -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r03av_$v.log 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/r03av_$v.log; exit 1; }
  python3 tools/rocpd_summary.py --stats /tmp/r03av_$v/run_results.db gpurun_out/r03av_${v}_kernel_stats.csv > /dev/null
  echo "$v: $(grep -E 'greedy_step|lm_head_kernel|embed' gpurun_out/r03av_${v}_kernel_stats.csv | tr '\n' ' ')" | tee -a gpurun_out/r03av_sampler_ab.txt
done
