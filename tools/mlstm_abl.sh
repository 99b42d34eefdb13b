#!/bin/bash
# mLSTM walk ablations (csrc/mlstm.hip SC_ML_ABL bits): build variants of the library under
# abl_build/ml<v>/ and time each with tools/mlstm_bench.py (SC_LIB_PATH).
# usage: tools/mlstm_abl.sh build | run   [variants, default below]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
V=${ML_ABL_SET:-"1 2 4 8 16 32 64 128 256 512"}
if [ "$1" = build ]; then
  for v in $V; do
    make -s -C "$R/statecatcher_amd/csrc" -j8 OUT="$R/abl_build/ml$v/libstatecatcher_hip.so" \
      BUILD="$R/abl_build/ml$v/obj" EXTRA="-DSC_ML_ABL=$v" lib
  done
  exit 0
fi
echo "== baseline"
timeout -k 10 100 python3 -u "$R/tools/mlstm_bench.py" --reps 10
for v in $V; do
  echo "== SC_ML_ABL=$v"
  SC_LIB_PATH="$R/abl_build/ml$v/libstatecatcher_hip.so" timeout -k 10 100 python3 -u "$R/tools/mlstm_bench.py" --reps 10
done
