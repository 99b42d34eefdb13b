#!/bin/bash
# A/B timing on the GPU box: tools/run_ab.sh <out-name> "<probe command>" <variant>...
# runs the probe with the in-tree library ("cur") and each tools/ab/<variant> library, in turn,
# twice around; output in gpurun_out/<out-name>.log
set -o pipefail
N=$1; CMD=$2; shift 2
O=gpurun_out/$N.log; mkdir -p gpurun_out; : > "$O"
for rnd in 1 2; do
  for v in cur "$@"; do
    echo "== $v (round $rnd)" >> "$O"
    if [ "$v" = cur ]; then L=""; else L=$PWD/tools/ab/$v/libstatecatcher_hip.so; fi
    SC_LIB_PATH=$L timeout -k 10 150 $CMD >> "$O" 2>&1 || { echo "FAILED rc=$?" >> "$O"; exit 1; }
  done
done
