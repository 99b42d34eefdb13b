#!/bin/bash
# Round-6 batch: GEMM + LN-fold + DDP tests, then the in-step A/B of the gate-forward variants
# (default library / SC_TN_FWD=2 / SC_LN_FOLD=2), alternated twice.  Each step has its own limit.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${TAG:-r6f}
timeout -k 10 900 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread \
  ${TESTS:-tests/test_gpu_ln_fold.py tests/test_gpu_ddp.py} > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_tests.log; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | cut -c1-150
[ -n "$NOAB" ] && exit $rc
for rnd in 1 2; do
  for v in base tn2 fold2; do
    case $v in
      base) E="";;
      tn2) E="SC_TN_FWD=2";;
      fold2) E="SC_LN_FOLD=2";;
    esac
    env $E timeout -k 10 300 python3 bench.py --cpu-baseline off > gpurun_out/${TAG}_ab_${v}_$rnd.json \
      2> gpurun_out/${TAG}_ab_${v}_$rnd.err || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_ab_${v}_$rnd.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d.get('kernels',{}); print(sys.argv[1], d['value'], d['ms_per_step'], {n: v.get('avg_us') for n, v in k.items() if 'gemm' in n or 'ln' in n or 'scan' in n})" gpurun_out/${TAG}_ab_${v}_$rnd.json
  done
done
exit $rc
