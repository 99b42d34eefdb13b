#!/bin/bash
# A/B libraries for the one-wave-per-SIMD TN kernels, only tn_gemm.hip recompiled:
#   tnf0: SC_TNW_FENCE=0 (the round-6 code as first measured), tnf1: the fenced fragment wait,
#   tnil: fenced + fragment reads interleaved with the MFMAs (SC_TNW_IL=1)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/statecatcher_amd/csrc
OBJS=$(ls $R/build/csrc/*.o | grep -v tn_gemm.o)
for spec in "tnf0:-DSC_TNW_FENCE=0" "tnf1:" "tnil:-DSC_TNW_IL=1"; do
  v=${spec%%:*}; f=${spec#*:}
  mkdir -p $R/tools/ab/$v
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$C -DSC_TNW_AB=1 $f \
    -c $C/tn_gemm.hip -o $R/tools/ab/$v/tn_gemm.o &
done
wait
for v in tnf0 tnf1 tnil; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $R/tools/ab/$v/tn_gemm.o \
    -o $R/tools/ab/$v/libstatecatcher_hip.so
done
