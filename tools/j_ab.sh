#!/bin/bash
# Fused-joiner backward A/B: the RNN-T joiner parity tests on the shipped library, then
# tools/joint_probe.py (C5 lattice, B = 32) alternating the shipped library and the variants
# built by tools/ab_build.sh under tools/ab/<name>/.
#   TAG=r5j VARIANTS="jd2" bash tools/j_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-j}
VARIANTS=${VARIANTS:-jd2}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_rnnt_joint.py tests/test_gpu_c5.py > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rnd in 1 2; do
  for v in cur $VARIANTS; do
    if [ "$v" = cur ]; then L=""; else L=$R/tools/ab/$v/libstatecatcher_hip.so; fi
    echo "== $v ($rnd)"
    SC_LIB_PATH=$L timeout -k 10 120 python3 -u tools/joint_probe.py 32 3 || exit $?
  done
done
