#!/bin/bash
# Round-5 focused GPU run: the given test files (default: the changed areas), then optionally
# (AB=1) the LN-fold A/B bench pair, (DRIFT=1) the same-box drift A/B.  Every GPU step has its
# own time limit; the first failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5}
TESTS=${TESTS:-"tests/test_gpu_ln_fold.py tests/test_gpu_ddp.py"}
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 200 --timeout-method thread $TESTS \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$AB" ]; then
  for rnd in 1 2; do
    for v in 1 0; do
      SC_LN_FOLD=$v timeout -k 10 300 python3 bench.py --cpu-baseline off > gpurun_out/${TAG}_ab_fold${v}_$rnd.json \
        2> gpurun_out/${TAG}_ab_fold${v}_$rnd.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_ab_fold${v}_$rnd.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], d['ms_per_step'], {k: v['avg_us'] for k, v in d['kernels'].items()})" gpurun_out/${TAG}_ab_fold${v}_$rnd.json
    done
  done
fi
if [ -n "$DRIFT" ]; then bash tools/drift_ab.sh $TAG; fi
if [ -n "$TNABL" ]; then
  for v in cur tn4 tn3 tn1; do
    echo "== $v"
    if [ "$v" = cur ]; then L=""; else L=$R/tools/ab/$v/libstatecatcher_hip.so; fi
    SC_LIB_PATH=$L timeout -k 10 200 python3 -u tools/tn_bench.py --tm 256 > gpurun_out/${TAG}_tn_$v.log 2>&1 \
      || { echo "tn bench failed"; tail -5 gpurun_out/${TAG}_tn_$v.log; exit 1; }
    grep -i "layer-0" gpurun_out/${TAG}_tn_$v.log
  done
fi
