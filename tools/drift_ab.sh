#!/bin/bash
# Same-box A/B of the round-1 tree (0318d98), the round-3 tree (7f900c4) and HEAD (verdict r4
# item 6).  The old trees are extracted and built by tools/ab_trees.sh into tools/ab/tree_r{1,3}.
#   tools/drift_ab.sh TAG      -> gpurun_out/drift_TAG.jsonl (one bench line per run, labelled)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r5}
O=$R/gpurun_out/drift_$TAG.jsonl
mkdir -p "$R/gpurun_out"; : > "$O"
run() {   # label dir args...
  local label=$1 dir=$2; shift 2
  echo "== $label $*"
  local line
  line=$(cd "$dir" && timeout -k 10 300 python3 bench.py --cpu-baseline off "$@" 2> "$R/gpurun_out/drift_${TAG}_err.log") \
    || { echo "FAILED $label rc=$?"; tail -20 "$R/gpurun_out/drift_${TAG}_err.log"; exit 1; }
  echo "{\"label\": \"$label\", \"args\": \"$*\", \"line\": $line}" >> "$O"
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'])" "$line"
}
for rnd in 1 2; do
  run head "$R" --steps 20 --warmup 5
  run head_bf16head "$R" --steps 20 --warmup 5 --output-head bf16
  run r1 "$R/tools/ab/tree_r1" --steps 20 --warmup 5
  run r3 "$R/tools/ab/tree_r3" --steps 20 --warmup 5
done
for rnd in 1 2; do
  for w in rnnt xlstm; do
    run head_$w "$R" --workload $w --steps 8 --warmup 4
    run r3_$w "$R/tools/ab/tree_r3" --workload $w --steps 8 --warmup 4
  done
done
