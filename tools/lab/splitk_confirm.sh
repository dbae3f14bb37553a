#!/bin/bash
# A/B of the fc2 split-K geometry: kernel alone (alternating) and the whole bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
# the override is compiled into lab builds only:
#   make -C kotoba-whisper_amd/csrc EXTRA=-DKW_LAB_OVERRIDES BUILD=build_lab OUT=../kwhisper/libkwhisper_lab.so
export KWHISPER_LIB="${KWHISPER_LIB:-$PWD/kotoba-whisper_amd/kwhisper/libkwhisper_lab.so}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for cfg in default 10,6 10,7; do
    if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=1280,5120,1,$cfg; fi
    echo -n "$cfg "
    timeout -k 10 120 python tools/kbench.py --reps 60 --only fc2_resid 2>/dev/null || exit 1
  done
done
for cfg in default 10,6 default 10,6; do
  if [ "$cfg" = default ]; then unset KW_DECLIN_GEO; else export KW_DECLIN_GEO=1280,5120,1,$cfg; fi
  echo -n "bench $cfg "
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(round(d['value'],1),round(d['decode_step_ms'],4))" || exit 1
done
