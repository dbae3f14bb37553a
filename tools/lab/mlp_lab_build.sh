#!/bin/bash
# Build a lab library (kotoba-whisper_amd/kwhisper/libkwhisper_lab.so) from the product sources copied to /tmp with a
# lab patch applied (default tools/lab/mlp_lab.diff: KW_MLP_LAB knobs in dec_mlp_kernel; tools/lab/fc2_rowsplit.diff:
# KW_DECLIN_ROWSPLIT=2), compiled under KW_LAB_OVERRIDES, so the product sources -- and the kernel-source hash the
# committed PMC profiles carry -- stay untouched.   bash tools/lab/mlp_lab_build.sh [patch]
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
T=/tmp/kw_mlp_lab_src
rm -rf "$T"
mkdir -p "$T/kotoba-whisper_amd" "$T/include"
cp -r "$ROOT/kotoba-whisper_amd/csrc" "$T/kotoba-whisper_amd/csrc"
rm -rf "$T/kotoba-whisper_amd/csrc/build" "$T/kotoba-whisper_amd/csrc/build_lab"
cp "$ROOT/include/kwhisper.h" "$T/include/"
PATCH="$(realpath "${1:-$ROOT/tools/lab/mlp_lab.diff}")"
(cd "$T" && patch -p1 < "$PATCH")
make -C "$T/kotoba-whisper_amd/csrc" -j8 EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab \
  OUT="$ROOT/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so" TORCH_OUT="$ROOT/kotoba-whisper_amd/kwhisper/libkwhisper_torch_lab.so"
