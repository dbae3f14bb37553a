# r03ab lab: the pair cross-attention with 7 chunks and a short last chunk (lab build -DKW_ROW_NS=7,
# KW_XA_CHUNK=<keys>: the final chunk's compute is the exposed tail) vs product (6 x 250)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
LAB="KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so"
for r in 1 2; do
  echo -n "base "; timeout -k 10 120 python tools/kbench.py --reps 40 --only cross_attn,xq_cross 2>/dev/null || exit 1
  for c in 248 240 224; do
    echo -n "lab$c "; env $LAB KW_XA_CHUNK=$c timeout -k 10 120 python tools/kbench.py --reps 40 --only cross_attn,xq_cross 2>/dev/null || exit 1
  done
done
