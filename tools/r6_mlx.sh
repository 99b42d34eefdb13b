#!/bin/bash
# mLSTM backward with each batch row's heads on one XCD (default build) against the identity
# mapping (tools/ab/mlx0, SC_ML_XCDH=0): the C4 tests, FETCH / WRITE per launch, and the C4 step
# alternated twice.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mlstm.py tests/test_gpu_xlstm_glue.py -q -x \
  --timeout 300 --timeout-method thread > $O/r6x_tests.log 2>&1
rc=$?; tail -3 $O/r6x_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for v in base mlx0; do
  L=$R/statecatcher_amd/libstatecatcher_hip.so; [ $v = mlx0 ] && L=$R/tools/ab/mlx0/libstatecatcher_hip.so
  for ctr in FETCH_SIZE WRITE_SIZE; do
    SC_LIB_PATH=$L timeout -k 10 240 rocprofv3 --pmc $ctr -f csv --kernel-include-regex "mlstm_bw" \
      -d $O/mlx_${v}_$ctr -o run -- python3 $R/bench.py --workload xlstm --steps 1 --warmup 1 \
      --cpu-baseline off > $O/mlx_${v}_$ctr.log 2>&1 || exit 1
    find $O/mlx_${v}_$ctr -type f ! -name "*counter_collection.csv" -delete
  done
done
cd $R
for rnd in 1 2; do
  for v in base mlx0; do
    L=$R/statecatcher_amd/libstatecatcher_hip.so; [ $v = mlx0 ] && L=$R/tools/ab/mlx0/libstatecatcher_hip.so
    SC_LIB_PATH=$L timeout -k 10 300 python3 -u bench.py --workload xlstm --cpu-baseline off \
      > $O/r6x_${v}_$rnd.json 2> $O/r6x_${v}_$rnd.err || exit 1
    python3 - $O/r6x_${v}_$rnd.json $v $rnd <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], {k: v.get("avg_us") for k, v in d.get("kernels", {}).items() if "mlstm" in k})
PY
  done
done
