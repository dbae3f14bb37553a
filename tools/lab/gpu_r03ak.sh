# r03ak lab: LM head weights by default-policy (MALL-allocating) loads (lab build -DKW_LMH_CACHED) vs non-temporal:
# the 133 MB matrix can stay in the 256 MB Infinity Cache between decode steps when every other stream is nt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in base lab; do
    if [ $v = base ]; then unset KWHISPER_LIB KWHISPER_TORCH_LIB; else export KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_lmh.json 2> gpurun_out/ab_lmh.err || { echo "FAIL $v"; tail -5 gpurun_out/ab_lmh.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_lmh.json')); print('$v', round(d['value'],1), 'step', round(d['decode_step_ms'],4), 'lm_head', d['decode_kernel_us']['lm_head'], 'xq_cross', d['decode_kernel_us']['xq_cross'])"
  done
done
