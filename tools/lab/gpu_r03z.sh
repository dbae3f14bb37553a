# r03z lab: encoder GEMM epilogue with non-temporal bf16 stores (lab build -DKW_GEMM_NT_STORE) vs product
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
LAB="KWHISPER_LIB=$PWD/build_lab/libkwhisper.so KWHISPER_TORCH_LIB=$PWD/build_lab/libkwhisper_torch.so"
for r in 1 2 3; do
  echo -n "base "; timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null || exit 1
  echo -n "lab  "; env $LAB timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null || exit 1
done
