#!/bin/bash
# Run GPU steps in order on the box, each under its own time limit; an ordinary failure (a failing test, exit 1)
# moves on to the next step, but a time limit, an abort or a signal (exit 124 / 134 / 137 / 139 / > 128) ends the
# call there: no further GPU work after a step that may have left the GPU in a bad state.
#   bash tools/gpu_steps.sh "<seconds> <log> <command...>" ...
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
status=0
for step in "$@"; do
  read -r secs log cmd <<< "$step"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$log" 2>&1
  rc=$?
  echo "[step] rc=$rc $log: $cmd" | cut -c1-200
  tail -4 "gpurun_out/$log"
  if [ $rc -ne 0 ]; then status=1; fi
  if [ $rc -ge 124 ]; then echo "[step] stopping: rc $rc"; exit $rc; fi
done
exit $status
