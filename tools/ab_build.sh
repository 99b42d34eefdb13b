#!/bin/bash
# Build an A/B variant of the C-ABI library into tools/ab/<name>/ (shipped to the GPU box with
# the tree; load it with SC_LIB_PATH=tools/ab/<name>/libstatecatcher_hip.so).
#   tools/ab_build.sh <name> "<EXTRA flags>" [source dir (default statecatcher_amd/csrc)]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; X=$2; SRC=${3:-$R/statecatcher_amd/csrc}
mkdir -p "$R/tools/ab/$N"
make -s -C "$SRC" -j8 ROOT="$R" OUT="$R/tools/ab/$N/libstatecatcher_hip.so" BUILD="/tmp/ab_build_$N" \
     EXTRA="$X" lib
