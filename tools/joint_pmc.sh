#!/bin/bash
# Kernel trace + SQ counters of the fused joiner at C5 (tools/joint_probe.py), separate passes.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/jpmc; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d "$O/kt" -o run -- python3 "$R/tools/joint_probe.py" 32 1 > "$O/kt.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex joint_bwd -f csv -d "$O/p1" -o run -- python3 "$R/tools/joint_probe.py" 32 1 > "$O/p1.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex joint_bwd -f csv -d "$O/p2" -o run -- python3 "$R/tools/joint_probe.py" 32 1 > "$O/p2.log" 2>&1
find "$O" -type f \( -name "*.db" -o -name "*agent_info*" -o -name "*_trace.csv" \) -delete
echo ok
