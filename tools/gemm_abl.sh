#!/bin/bash
# Variant builds of the full library for gemm.hip experiments: SC_GEMM_ABL ablation bitmask
# (ABL list) and extra flags (EXTRA, e.g. -DSC_GEMM_SLOTS=4), into abl_build/gemm_abl$v$TAG.so;
# time each on the GPU box with: SC_LIB_PATH=abl_build/gemm_abl$v$TAG.so python tools/gemm_bench.py
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/abl_build
mkdir -p "$O/objs"
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$R/statecatcher_amd/csrc $EXTRA"
objs=""
for f in "$R"/build/csrc/*.o; do
  b=$(basename "$f")
  [ "$b" = gemm.o ] || objs="$objs $f"
done
for v in ${ABL:-0 1 2 4}; do
  (/opt/rocm/bin/hipcc $FL -DSC_GEMM_ABL=$v -c "$R/statecatcher_amd/csrc/gemm.hip" -o "$O/objs/gemm$v$TAG.o" &&
   /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs "$O/objs/gemm$v$TAG.o" -o "$O/gemm_abl$v$TAG.so") &
done
wait
ls "$O"
