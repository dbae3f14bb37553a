#!/bin/bash
# r05e: config-4 multi-pass scan of the fixture model (numpy weights) on the HIP log-mel, bf16 and fp32, with the
# features of every multi-pass clip; config 4 measured on the same model (dynamic schedule).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/find_multipass.py --n-clips 1768 --dtype bfloat16 --weights numpy --out gpurun_out/r05e_mp_bf16.json --features-out gpurun_out/r05e_mp_bf16_features.npz > gpurun_out/r05e_mp_bf16.log 2>&1 || { tail -5 gpurun_out/r05e_mp_bf16.log; exit 1; }
tail -1 gpurun_out/r05e_mp_bf16.log
timeout -k 10 600 python -u tools/find_multipass.py --n-clips 1768 --dtype float32 --weights numpy --out gpurun_out/r05e_mp_fp32.json --features-out gpurun_out/r05e_mp_fp32_features.npz > gpurun_out/r05e_mp_fp32.log 2>&1 || { tail -5 gpurun_out/r05e_mp_fp32.log; exit 1; }
tail -1 gpurun_out/r05e_mp_fp32.log
timeout -k 10 400 python tools/bench_configs.py --config 4 > gpurun_out/r05e_config4.json 2> gpurun_out/r05e_config4.err && python -c "import json; d=json.loads(open('gpurun_out/r05e_config4.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('value', 'padded_30s_value', 'seconds', 'dp_projection')}, d['batch_seek_passes'])"
