#!/bin/bash
# joint_bwd_pc_kernel (SC_JOINT_PC=1 build, tools/ab/jpc): the RNN-T joiner tests on that
# library, then tools/joint_probe.py shipped vs jpc, then the CTC wmax A/B (tools/ab/ctcw).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5pc}
SC_LIB_PATH=$R/tools/ab/jpc/libstatecatcher_hip.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 \
  --timeout-method thread tests/test_gpu_rnnt_joint.py tests/test_gpu_c5.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rnd in 1 2; do
  for v in cur jpc; do
    if [ "$v" = cur ]; then L=""; else L=$R/tools/ab/$v/libstatecatcher_hip.so; fi
    echo "== $v ($rnd)"
    SC_LIB_PATH=$L timeout -k 10 120 python3 -u tools/joint_probe.py 32 3 || exit $?
  done
done
for rnd in 1 2; do
  for v in cur ctcw; do
    if [ "$v" = cur ]; then L=""; else L=$R/tools/ab/$v/libstatecatcher_hip.so; fi
    echo "== $v ($rnd)"
    SC_LIB_PATH=$L timeout -k 10 120 python3 -u tools/scan_bench.py --only ctc --iters 20 || exit $?
  done
done
