#!/bin/bash
# Round-6 GPU runs: TESTS (pytest files, optional), then TN (the TN ablation set at tm 256),
# then CMD (any extra command).  Every GPU step has its own time limit; the first failure ends.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r6}
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TT:-900} python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread $TESTS \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "$TN" ]; then
  for v in $TN; do
    echo "== $v"
    if [ "$v" = cur ]; then L=""; else L=$R/tools/ab/$v/libstatecatcher_hip.so; fi
    SC_LIB_PATH=$L timeout -k 10 200 python3 -u tools/tn_bench.py --tm ${TM:-256} > gpurun_out/${TAG}_tn_$v.log 2>&1 \
      || { echo "tn bench failed"; tail -5 gpurun_out/${TAG}_tn_$v.log; exit 1; }
    cat gpurun_out/${TAG}_tn_$v.log
  done
fi
if [ -n "$CMD" ]; then
  timeout -k 10 ${CT:-600} bash -c "$CMD" > gpurun_out/${TAG}_cmd.log 2>&1
  rc=$?; tail -30 gpurun_out/${TAG}_cmd.log; exit $rc
fi
