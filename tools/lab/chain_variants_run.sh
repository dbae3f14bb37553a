#!/bin/bash
# Lab (not product): tools/lab/chain_lab.py over the builds of tools/lab/chain_variants.sh (on the GPU box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in "" xplain stplain both sleep20; do
  if [ -n "$v" ]; then export KWHISPER_LIB=$PWD/build_lab_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab_$v/libkwhisper_torch.so; fi
  echo "== ${v:-product}"
  timeout -k 10 120 python -u tools/lab/chain_lab.py --iters 10 2>/dev/null | tail -1 || exit 1
done
