#!/bin/bash
# TN GEMM ablation libraries built from the in-tree objects with only tn_gemm.hip recompiled
# (SC_TN_ABL bits: 1 no MFMA, 2 no DMA after the prologue, 4 no output stores).
# usage: tools/tn_abl2.sh 4 6 ...   -> tools/ab/tn<v>/libstatecatcher_hip.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/statecatcher_amd/csrc
OBJS=$(ls $R/build/csrc/*.o | grep -v tn_gemm.o)
for v in "$@"; do
  mkdir -p $R/tools/ab/tn$v
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C -DSC_TN_ABL=$v \
    -c $C/tn_gemm.hip -o $R/tools/ab/tn$v/tn_gemm.o
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $R/tools/ab/tn$v/tn_gemm.o \
    -o $R/tools/ab/tn$v/libstatecatcher_hip.so
done
