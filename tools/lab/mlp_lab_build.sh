#!/bin/bash
# Build the r04 fused-MLP lab library (kotoba-whisper_amd/kwhisper/libkwhisper_lab.so): the product sources copied to
# /tmp with tools/lab/mlp_lab.diff applied (KW_MLP_LAB knobs in dec_mlp_kernel, compiled under KW_LAB_OVERRIDES), so
# the product declin.hip -- and the kernel-source hash the committed PMC profiles carry -- stay untouched.
set -e
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
T=/tmp/kw_mlp_lab_src
rm -rf "$T"
mkdir -p "$T/kotoba-whisper_amd" "$T/include"
cp -r "$ROOT/kotoba-whisper_amd/csrc" "$T/kotoba-whisper_amd/csrc"
rm -rf "$T/kotoba-whisper_amd/csrc/build" "$T/kotoba-whisper_amd/csrc/build_lab"
cp "$ROOT/include/kwhisper.h" "$T/include/"
(cd "$T" && patch -p1 < "$ROOT/tools/lab/mlp_lab.diff")
make -C "$T/kotoba-whisper_amd/csrc" -j8 EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab \
  OUT="$ROOT/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so" TORCH_OUT="$ROOT/kotoba-whisper_amd/kwhisper/libkwhisper_torch_lab.so"
