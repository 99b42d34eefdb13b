#!/bin/bash
# Round-6 combined call: GEMM tests, tnw/tnw32 bench + ablations, LN-fold / DDP / parity tests,
# then the in-step A/B (tools/r6_batch.sh).  Each step has its own limit; failures are reported
# and the next independent step still runs unless the GPU itself faulted.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${TAG:-r6g}
timeout -k 10 600 python3 -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_gpu_gemm.py \
  > gpurun_out/${TAG}_gemm.log 2>&1; rc=$?; echo "gemm tests rc=$rc"; tail -3 gpurun_out/${TAG}_gemm.log
case $rc in 124|134|137|139) exit $rc;; esac
TAG=$TAG bash tools/r6_tnw.sh > gpurun_out/${TAG}_tnw.log 2>&1; rc=$?; echo "tnw rc=$rc"; cat gpurun_out/${TAG}_tnw.log
case $rc in 124|134|137|139) exit $rc;; esac
TAG=$TAG TESTS="tests/test_gpu_ln_fold.py tests/test_gpu_parity_step.py tests/test_gpu_ddp.py" bash tools/r6_batch.sh
