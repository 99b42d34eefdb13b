#!/bin/bash
# Ablation builds of the streaming frame kernels (SC_FRAME_ABL bitmask, lucy_frame.hip) as whole
# libraries under abl_build/frame<N>.so; time each on the box with SC_LIB_PATH=... (results are
# wrong by construction: timing only).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -C "$R/statecatcher_amd/csrc" -j8 >/dev/null
O=$R/abl_build
mkdir -p "$O"
B=$R/build/csrc
OBJS=$(ls $B/*.o | grep -v '/lucy_frame.o$')
for v in ${ABL:-0 1 2 4 8 12}; do
  (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -I$R/statecatcher_amd/csrc \
     -DSC_FRAME_ABL=$v -c "$R/statecatcher_amd/csrc/lucy_frame.hip" -o "$O/frame$v.o" &&
   /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS "$O/frame$v.o" -o "$O/frame$v.so") &
done
wait
ls "$O"/frame*.so
