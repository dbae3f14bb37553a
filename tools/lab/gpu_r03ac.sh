# r03ac lab: the in-launch hand-off polls' sleep (KW_POLL_SLEEP x 64 cycles between polls): product (1) vs 4, 16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  for v in base s4 s16; do
    if [ $v = base ]; then unset KWHISPER_LIB KWHISPER_TORCH_LIB; else export KWHISPER_LIB=$PWD/build_$v/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_$v/libkwhisper_torch.so; fi
    echo -n "$v "; timeout -k 10 120 python tools/kbench.py --reps 40 --only cross_attn,xq_cross,qkv_self --self-t 64,132 2>/dev/null || exit 1
  done
done
