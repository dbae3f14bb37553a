#!/bin/bash
# r06aa: kw_dec_qkv_self_o -- the self block's out-projection fused into its launch as a consumer (160 workgroups
# after the pairs, weights loaded at launch, per-row-half arrival counts): tests (bitwise vs the two launches,
# tokens), kbench (qkv_self + o_resid vs qkv_self_o), bench A/B on one library (KW_FUSE_SELF_O=1 / 0).
# Ran against the round-6 fusion sources, since reverted (slower: profiles/r06aa_self_o_fusion_ab.txt);
# the entry point, the KW_FUSE_SELF_O switch and the tests it names are not in the tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_generate.py -x -v --timeout 120 --timeout-method thread -k "qkv_self_o or self_o_tokens or qkv or xq or fused or tokens_identical or handoff" > gpurun_out/r06aa_pytest.log 2>&1 && echo TESTS_OK && tail -1 gpurun_out/r06aa_pytest.log || { grep -E "FAILED|Error|assert" gpurun_out/r06aa_pytest.log | head -20; exit 1; }
for r in 1 2; do
  timeout -k 10 150 python tools/kbench.py --only o_resid,qkv_self,qkv_self_o > gpurun_out/r06aa_kb.json 2> gpurun_out/r06aa_kb.err && echo "kb $(tail -c 300 gpurun_out/r06aa_kb.json)" || { tail -5 gpurun_out/r06aa_kb.err; exit 1; }
done
for r in 1 2; do
  for v in 1 0; do
    KW_FUSE_SELF_O=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r06aa_bench_$v.json 2> gpurun_out/r06aa_bench.err || { echo "FAIL $v"; tail -5 gpurun_out/r06aa_bench.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r06aa_bench_$v.json')); print('fuse_self_o=$v', round(d['value'],1), round(d['decode_step_ms'],3))"
  done
done
