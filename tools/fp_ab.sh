#!/bin/bash
# RCCL-footprint A/B on one GPU (verdict r4 item 1): the C2 bench with no side stream, then with
# bench.py --rccl-footprint WGS:SLEEP (persistent copy workgroups on a side stream during the
# backward, the bytes of an 8-GPU ring all-reduce), alternated twice.
#   TAG=r5 bash tools/fp_ab.sh   -> gpurun_out/fp_TAG.jsonl
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5}
O=gpurun_out/fp_$TAG.jsonl; : > "$O"
for rnd in 1 2; do
  for fp in off 16:1 32:0 32:1 64:1; do
    if [ $fp = off ]; then A=""; else A="--rccl-footprint $fp"; fi
    line=$(timeout -k 10 300 python3 bench.py --cpu-baseline off --steps 20 --warmup 5 $A 2> gpurun_out/fp_${TAG}_err.log) \
      || { echo "FAILED $fp"; tail -20 gpurun_out/fp_${TAG}_err.log; exit 1; }
    echo "{\"footprint\": \"$fp\", \"line\": $line}" >> "$O"
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(sys.argv[1], d['value'], d['ms_per_step'])" "$fp" "$line"
  done
done
