#!/bin/bash
# ctc_grad2_kernel (default) against ctc_grad_kernel (tools/ab/grad1): bitwise A/B of losses and
# gradients, then timing (tools/scan_bench.py --only ctc, interleaved), then the CTC GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5m}
timeout -k 10 200 python3 -u tools/ctc_grad_ab.py save gpurun_out/${TAG}_g2.pt > gpurun_out/${TAG}_ab.log 2>&1 || exit $?
SC_LIB_PATH=$R/tools/ab/grad1/libstatecatcher_hip.so timeout -k 10 200 python3 -u tools/ctc_grad_ab.py save gpurun_out/${TAG}_g1.pt >> gpurun_out/${TAG}_ab.log 2>&1 || exit $?
python3 tools/ctc_grad_ab.py compare gpurun_out/${TAG}_g2.pt gpurun_out/${TAG}_g1.pt; rc=$?
rm -f gpurun_out/${TAG}_g1.pt gpurun_out/${TAG}_g2.pt
[ $rc -eq 0 ] || exit $rc
for rnd in 1 2; do
  for v in cur grad1; do
    if [ $v = cur ]; then L=""; else L=$R/tools/ab/$v/libstatecatcher_hip.so; fi
    echo "== $v ($rnd)"
    SC_LIB_PATH=$L timeout -k 10 120 python3 -u tools/scan_bench.py --only ctc --iters 20 || exit $?
  done
done
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ctc.py \
  tests/test_gpu_ctc_head.py tests/test_gpu_parity_step.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log; exit $rc
