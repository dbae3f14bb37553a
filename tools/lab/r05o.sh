#!/bin/bash
# r05o: where the bench's encoder time goes -- kernel-trace timelines of the one-pass (--streams 1) and the two-row-block
# (--streams 2) large-v3 B = 32 encoder (tools/enc_pass.py), summarised by tools/lab/enc_timeline.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 1 2; do
  rm -rf /tmp/r05o_s$s
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d /tmp/r05o_s$s -o run -- python3 tools/enc_pass.py --streams $s --reps 3 > gpurun_out/r05o_s$s.log 2>&1 || exit 1
  f=$(ls /tmp/r05o_s$s/*kernel_trace.csv /tmp/r05o_s$s/*/*kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/lab/enc_timeline.py "$f" > gpurun_out/r05o_timeline_s$s.json || exit 1
  cat gpurun_out/r05o_timeline_s$s.json
done
