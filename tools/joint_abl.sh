#!/bin/bash
# Fused-joiner backward ablations (csrc/rnnt.hip SC_JOINT_ABL bits): variants built under
# abl_build/j<v>/ (make ... EXTRA=-DSC_JOINT_ABL=<v> lib), each timed by tools/joint_probe.py.
# usage: JOINT_ABL_SET="1 2 4 8" tools/joint_abl.sh
R=$(cd "$(dirname "$0")/.." && pwd)
V=${JOINT_ABL_SET:-"1 2 4 8"}
echo "== shipped"
timeout -k 10 120 python3 -u "$R/tools/joint_probe.py" 32 3 || exit $?
for v in $V; do
  echo "== SC_JOINT_ABL=$v"
  SC_LIB_PATH="$R/abl_build/j$v/libstatecatcher_hip.so" timeout -k 10 120 python3 -u "$R/tools/joint_probe.py" 32 3 || exit $?
done
