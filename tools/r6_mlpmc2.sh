#!/bin/bash
# mLSTM backward: FETCH_SIZE / WRITE_SIZE of the build without the dq / dk / dv stores
# (SC_ML_ABL=262144) against the default build: partial-line gradient stores that make the
# L2 read their lines from HBM show up as FETCH that no operand accounts for.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {   # tag lib counter
  SC_LIB_PATH=$2 timeout -k 10 240 rocprofv3 --pmc $3 -f csv --kernel-include-regex "mlstm_bw" \
    -d $O/mlpmc_$1_$3 -o run -- python3 $R/bench.py --workload xlstm --steps 1 --warmup 1 \
    --cpu-baseline off > $O/mlpmc_$1_$3.log 2>&1 || return 1
  find $O/mlpmc_$1_$3 -type f ! -name "*counter_collection.csv" -delete
  echo "$1 $3 done"
}
run ml262144 $R/tools/ab/ml262144/libstatecatcher_hip.so FETCH_SIZE || exit 1
run ml262144 $R/tools/ab/ml262144/libstatecatcher_hip.so WRITE_SIZE || exit 1
