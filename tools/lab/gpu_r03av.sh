# r03av lab: greedy sampler with one arrival count over all B x NSPLIT workgroups (lab build in build_lab/) vs the
# per-row count + second count of the in-tree library: bench A/B in three alternating rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base lab; do
    if [ $v = base ]; then unset KWHISPER_LIB KWHISPER_TORCH_LIB; else export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_smp.json 2> gpurun_out/ab_smp.err || { echo "FAIL $v"; tail -5 gpurun_out/ab_smp.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_smp.json')); print('$v', round(d['value'],1), 'step', round(d['decode_step_ms'],4))" | tee -a gpurun_out/r03av_sampler_ab.txt
  done
done
