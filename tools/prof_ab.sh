#!/bin/bash
# rocprofv3 kernel-trace stats of the C2 bench under two bench.py flag sets, for an A/B of
# where a change's time goes.  usage: tools/prof_ab.sh TAG "flags A" "flags B"
# (a NAME=value word in a flag set is exported to that side's environment instead)
# Outputs: gpurun_out/prof_TAG_{a,b}/run_kernel_stats.csv (other profiler files deleted).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for side in a b; do
  if [ $side = a ]; then W=$2; else W=$3; fi
  F=""
  for w in $W; do
    case $w in
      --*) F="$F $w" ;;
      *=*) export "$w" ;;
      *) F="$F $w" ;;
    esac
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_${TAG}_$side" -o run -- \
    python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline off $F > "$O/prof_${TAG}_$side.json" 2> "$O/prof_${TAG}_$side.err"
  find "$O/prof_${TAG}_$side" -type f ! -name "*kernel_stats.csv" -delete
  for w in $W; do case $w in --*) ;; *=*) unset "${w%%=*}" ;; esac; done
done
echo done
