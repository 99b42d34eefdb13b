#!/bin/bash
# L2 / L1 counters of the LN-fold TN kernel and hipBLASLt's gate-forward kernel in one process
# (tools/tn_bench.py --ln --shapes 0): one rocprofv3 --pmc pass per counter group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "FETCH_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -f csv -d $O/tnpmc_$i -o run -- \
    python3 $R/tools/tn_bench.py --ln --shapes 0 > $O/tnpmc_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  find $O/tnpmc_$i -type f ! -name "*counter_collection.csv" -delete
  echo "pass $i ($grp) done"
done
