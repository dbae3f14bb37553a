#!/bin/bash
# Submit one gpurun command, re-submitting it only while the pool reports no free box / an infrastructure
# transient (nothing ran, nothing charged); any verdict from an actual run is final.  Usage:
#   tools/gpurun_wait.sh <timeout-seconds> '<command>'
t="$1"; shift
for attempt in $(seq 1 40); do
  out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -q "status=transient"; then
    echo "[gpurun_wait] attempt $attempt: transient, waiting" >&2
    sleep 150
    continue
  fi
  echo "$out" | tail -30
  exit $rc
done
echo "[gpurun_wait] gave up after 40 transient attempts" >&2
exit 3
