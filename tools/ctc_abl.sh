#!/bin/bash
# Ablation builds of the CTC kernels (SC_CTC_ABL bitmask, ctc.hip) as whole libraries under
# abl_build/ctc<N>.so; time each on the box with SC_LIB_PATH=... tools/scan_bench.py --only ctc.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -C "$R/statecatcher_amd/csrc" -j8 >/dev/null
O=$R/abl_build
mkdir -p "$O"
B=$R/build/csrc
OBJS=$(ls $B/*.o | grep -v '/ctc.o$')
for v in ${ABL:-0 1 2 4 7}; do
  (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$R/statecatcher_amd/csrc \
     -DSC_CTC_ABL=$v $EXTRA_DEF -c "$R/statecatcher_amd/csrc/ctc.hip" -o "$O/ctc$v$SUF.o" &&
   /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS "$O/ctc$v$SUF.o" -o "$O/ctc$v$SUF.so") &
done
wait
ls "$O"/ctc*.so
