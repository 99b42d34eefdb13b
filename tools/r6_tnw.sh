#!/bin/bash
# tnw / tnw32 (tile_m 1 / 2 / 3) against the library at the gate-forward and input-gradient
# shapes, then the ablation builds of tools/tn_abl2.sh on tile_m 2.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${TAG:-r6e}
for tm in 2 3 1; do
  echo "== tm $tm"
  timeout -k 10 150 python3 -u tools/tn_bench.py --tm $tm --shapes 0,2,4 --nolib 2>&1 | grep -v amdgpu.ids || exit 1
done
for v in tn1 tn2 tn4; do
  echo "== abl $v (tm 2)"
  SC_LIB_PATH=$PWD/tools/ab/$v/libstatecatcher_hip.so timeout -k 10 150 python3 -u tools/tn_bench.py --tm 2 --shapes 0 --nolib 2>&1 | grep -v amdgpu.ids || exit 1
done
