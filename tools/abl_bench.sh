#!/bin/bash
# Build ablation variants of the scan library (SC_ABL bitmask, lucy_scan.hip) into abl_build/ (git-ignored, travels to the box)
# and the abl_bench harness.  Run abl_build/abl_bench abl_build/*.so on the GPU box.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/abl_build
mkdir -p "$O"
CXX="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$R/statecatcher_amd/csrc"
for v in ${ABL:-0 1 2 4 8 3 15}; do
  $CXX -DSC_ABL=$v -shared "$R/statecatcher_amd/csrc/lucy_scan.hip" "$R/statecatcher_amd/csrc/capi.cpp" \
    -o "$O/abl$v.so" &
done
$CXX "$R/tools/abl_bench.cpp" -o "$O/abl_bench" -ldl &
wait
ls "$O"
