#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that ends in a
# fault, abort, segfault, timeout or kill (exit 124/134/137/139 or >128), so nothing more runs on a
# GPU that may be unhealthy.  An ordinary failure (e.g. a failing assertion, exit 1) lets the
# next step run.  usage: tools/gpu_steps.sh "<seconds> <log> <cmd...>" ...
rc_all=0
for step in "$@"; do
  secs=${step%% *}; rest=${step#* }
  log=${rest%% *}; cmd=${rest#* }
  timeout -k 10 "$secs" bash -c "$cmd" > "$log" 2>&1
  rc=$?
  echo "step rc=$rc: $cmd" >> gpurun_out/steps.log
  if [ $rc -ge 124 ]; then echo "stopping after rc=$rc ($cmd)"; exit $rc; fi
  [ $rc -ne 0 ] && rc_all=$rc
done
exit $rc_all
