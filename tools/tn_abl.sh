#!/bin/bash
# TN GEMM ablations: build no-MFMA and no-DMA variants of the library under abl_build/ and time
# them with tools/tn_bench.py (SC_LIB_PATH).  usage: tools/tn_abl.sh build | run
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
if [ "$1" = build ]; then
  for v in 1 2; do
    make -s -C "$R/statecatcher_amd/csrc" -j8 OUT="$R/abl_build/tn$v/libstatecatcher_hip.so" \
      BUILD="$R/abl_build/tn$v/obj" EXTRA="-DSC_TN_ABL=$v"
  done
  exit 0
fi
for v in 1 2; do
  echo "== SC_TN_ABL=$v"
  SC_LIB_PATH="$R/abl_build/tn$v/libstatecatcher_hip.so" timeout -k 10 200 python3 -u "$R/tools/tn_bench.py" --tm 192
done
