#!/bin/bash
# Extract and build earlier trees for same-box A/B runs (tools/drift_ab.sh):
#   tools/ab_trees.sh r1:0318d98 r3:7f900c4
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for spec in "$@"; do
  n=${spec%%:*}; rev=${spec##*:}; d=$R/tools/ab/tree_$n
  rm -rf "$d"; mkdir -p "$d"
  git -C "$R" archive "$rev" statecatcher_amd include bench.py oracle | tar -x -C "$d"
  make -s -C "$d/statecatcher_amd/csrc" -j8 BUILD=/tmp/abtree_$n all
done
