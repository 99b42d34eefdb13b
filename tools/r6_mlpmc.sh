#!/bin/bash
# mLSTM backward per-operand FETCH: one FETCH_SIZE pass (and one WRITE_SIZE pass for the baseline)
# of the C4 bench step per build; a build without an operand's loads shows what that operand
# costs in fetched bytes (tools/mlstm_abl.sh build, copied to tools/ab/ml<v>).
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
run base $R/statecatcher_amd/libstatecatcher_hip.so FETCH_SIZE || exit 1
run base $R/statecatcher_amd/libstatecatcher_hip.so WRITE_SIZE || exit 1
for v in 4096 8192 16384 32768 65536 131072; do
  run ml$v $R/tools/ab/ml$v/libstatecatcher_hip.so FETCH_SIZE || exit 1
done
