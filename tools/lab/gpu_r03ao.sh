set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/lab/enc_parts_sweep.py > gpurun_out/r03ao_enc_parts.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r03ao_enc_parts.txt | tail -6; [ $rc -eq 0 ] &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03ao_bench.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/r03ao_bench.json')); print(round(d['value'],1), d['encoder_mfma'], d['decode_step_ms'])"
