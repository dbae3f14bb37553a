#!/bin/bash
# Lab A/B (not product): decode step with and without cross K/V warm-up reads (KW_KV_PREFETCH=wgs[,nt]).
# The knob and its kernel were removed after the negative result in profiles/r02g_lab_notes.md; kept as the record.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "" 256 512 128 "256,nt" ""; do
  KW_KV_PREFETCH=$cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab_pf.json 2> gpurun_out/ab_pf.err || { echo "FAIL $cfg"; tail -5 gpurun_out/ab_pf.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_pf.json')); print('pf=[$cfg]', round(d['value'],1), round(d['decode_step_ms'],3), d['decode_kernel_us'])"
done
