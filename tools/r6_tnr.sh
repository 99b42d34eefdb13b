#!/bin/bash
# Register-staged TN kernel (tnr, SC_TNR=1 build in tools/ab/tnr): plain (tile_m 2) at the gate
# forward and input-gradient shapes, and the LN-fold instance, against the library.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
L=$PWD/tools/ab/tnr/libstatecatcher_hip.so
echo "== tnr plain"
SC_LIB_PATH=$L timeout -k 10 150 python3 -u tools/tn_bench.py --tm 2 --shapes 0,2 --nolib 2>&1 | grep -v amdgpu.ids || exit 1
echo "== tnr LN"
SC_LIB_PATH=$L timeout -k 10 150 python3 -u tools/tn_bench.py --ln --shapes 0 --nolib 2>&1 | grep -v amdgpu.ids || exit 1
