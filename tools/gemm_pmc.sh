#!/bin/bash
# MFMA-busy counters of the C2 step's GEMMs (hipBLASLt / rocBLAS, wgrad_kernel, tn_kernel): one
# rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE), no other trace.
# usage: tools/gemm_pmc.sh TAG  ->  gpurun_out/gpmc_TAG/run_counter_collection.csv
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2}
O=$R/gpurun_out/gpmc_$TAG; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  --kernel-include-regex "Cijk|wgrad_kernel|tn_kernel" -f csv -d "$O" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-baseline off > "$O/run.log" 2>&1
find "$O" -type f ! -name "*counter_collection.csv" ! -name "run.log" -delete
echo ok
