#!/bin/bash
# Build a lab library (kotoba-whisper_amd/kwhisper/libkwhisper_lab.so) from the product sources copied to /tmp with
# tools/lab/lab_switches.diff applied -- the lab switches that used to sit in the product kernels behind #if (round 6,
# VERDICT r5 item 6): KW_LAB_MLP (the fused decode MLP kw_dec_mlp and its KW_MLP_LAB decomposition knobs),
# KW_LAB_OVERRIDES (KW_DECLIN_GEO / KW_DECLIN_ROWSPLIT / KW_GEMM_TILE environment overrides), KW_LMH_LAB /
# KW_LMH_BUFS / KW_LMH_MAX_ROWS (LM head decompositions), KW_GEMM_LAB (GEMM epilogue decompositions) and
# KW_BEAM_LAB_* (beam top-k sweeps) -- plus an optional second patch, compiled with the given defines, so the product
# sources (and the kernel-source hash the committed PMC profiles carry) stay untouched.
#   bash tools/lab/mlp_lab_build.sh ["-DKW_LAB_MLP -DKW_LAB_OVERRIDES ..."] [extra.diff]
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
T=/tmp/kw_mlp_lab_src
rm -rf "$T"
mkdir -p "$T/kotoba-whisper_amd" "$T/include" "$T/tools/lab"
cp -r "$ROOT/kotoba-whisper_amd/csrc" "$T/kotoba-whisper_amd/csrc"
rm -rf "$T/kotoba-whisper_amd/csrc/build" "$T/kotoba-whisper_amd/csrc/build_lab"
cp "$ROOT/include/kwhisper.h" "$T/include/"
cp "$ROOT/tools/lab/kw_mlp_lab.h" "$T/tools/lab/"
(cd "$T" && patch -p1 < "$ROOT/tools/lab/lab_switches.diff")
if [ -n "$2" ]; then
  PATCH="$(realpath "$2")"
  (cd "$T" && patch -p1 < "$PATCH")
fi
make -C "$T/kotoba-whisper_amd/csrc" -j8 EXTRA="${1:--DKW_LAB_OVERRIDES}" BUILD=build_lab \
  OUT="$ROOT/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so" TORCH_OUT="$ROOT/kotoba-whisper_amd/kwhisper/libkwhisper_torch_lab.so"
