# r03y lab: fc2 (split-K) with the activation slices staged by LDS-DMA (KW_DECLIN_XLDS_SPLIT, lab build) vs product
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LAB="KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so"
timeout -k 10 120 python tools/lab/fc2_out.py gpurun_out/fc2_base.pt &&
env $LAB KW_DECLIN_XLDS_SPLIT=1 timeout -k 10 120 python tools/lab/fc2_out.py gpurun_out/fc2_lab.pt &&
python -c "
import torch; a=torch.load('gpurun_out/fc2_base.pt'); b=torch.load('gpurun_out/fc2_lab.pt')
print('bitwise h', torch.equal(a['h'], b['h']), 'hb', torch.equal(a['hb'].view(torch.int16), b['hb'].view(torch.int16)))" || exit 1
for r in 1 2 3; do
  echo -n "base "; timeout -k 10 120 python tools/kbench.py --reps 40 --only fc2_resid,fc1_ln_gelu,o_resid 2>/dev/null || exit 1
  echo -n "lab  "; env $LAB KW_DECLIN_XLDS_SPLIT=1 timeout -k 10 120 python tools/kbench.py --reps 40 --only fc2_resid,fc1_ln_gelu,o_resid 2>/dev/null || exit 1
done
