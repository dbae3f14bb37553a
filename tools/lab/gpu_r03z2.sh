# r03z lab: bench encoder time with non-temporal GEMM stores: base vs all bf16 epilogues nt (build_lab) vs
# head-split + GELU epilogues only (build_lab2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in base lab lab2; do
    if [ $v = base ]; then unset KWHISPER_LIB KWHISPER_TORCH_LIB; else export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_nt.json 2> gpurun_out/ab_nt.err || { echo "FAIL $v"; tail -5 gpurun_out/ab_nt.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_nt.json')); print('$v', round(d['value'],1), 'enc_ms', round(d['encoder_mfma']['ms'],2), 'step', round(d['decode_step_ms'],3))"
  done
done
