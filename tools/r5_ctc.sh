#!/bin/bash
# CTC alpha-beta exchange A/B: the CTC GPU tests on the shipped library, then tools/scan_bench.py
# --only ctc alternating the shipped library (flag exchanges) and tools/ab/ctcb (barriers).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5c}
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ctc.py tests/test_gpu_ctc_head.py \
  tests/test_gpu_parity_step.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rnd in 1 2; do
  for v in cur ${CTC_VARIANTS:-ctc0}; do
    if [ "$v" = cur ]; then L=""; else L=$R/tools/ab/$v/libstatecatcher_hip.so; fi
    echo "== $v ($rnd)"
    SC_LIB_PATH=$L timeout -k 10 120 python3 -u tools/scan_bench.py --only ctc --iters 20 || exit $?
  done
done
