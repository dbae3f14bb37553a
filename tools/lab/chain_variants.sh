#!/bin/bash
# Lab (not product): build kw_dec_chain variants (lab macros) into build_lab_<name>/ (run here, on the CPU)
set -e
cd /root/repo/kotoba-whisper_amd/csrc
build() { make -j8 EXTRA="-DKW_LAB_OVERRIDES $2" BUILD=/root/repo/build_lab_$1/obj OUT=/root/repo/build_lab_$1/libkwhisper.so TORCH_OUT=/root/repo/build_lab_$1/libkwhisper_torch.so > /dev/null; }
build xplain "-DKW_CH_XLD=0"
build stplain "-DKW_CH_PLAIN_ST=1"
build both "-DKW_CH_XLD=0 -DKW_CH_PLAIN_ST=1"
build sleep20 "-DKW_CH_SLEEP=20"
