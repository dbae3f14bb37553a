# r03y lab: fc2 geometry sweep with split-K activations staged by LDS-DMA (lab build, KW_DECLIN_GEO=N,K,ncb,ktm,ks)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so KW_DECLIN_XLDS_SPLIT=1
for rep in 1 2; do
  for cfg in default 1280,5120,2,10,6 1280,5120,2,10,4 1280,5120,1,10,4 1280,5120,1,10,5 1280,5120,1,5,8 1280,5120,2,5,8 1280,5120,1,10,8 1280,5120,2,10,8; do
    if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=$cfg; fi
    echo -n "$cfg "
    timeout -k 10 120 python tools/kbench.py --reps 40 --only fc2_resid 2>/dev/null || exit 1
  done
done
