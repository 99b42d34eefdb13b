#!/bin/bash
# Round-5 focused GPU tests (the changed areas), then the same-box drift A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread \
  tests/test_gpu_ctc.py tests/test_gpu_rnnt_joint.py tests/test_gpu_rnnt.py tests/test_gpu_mlstm.py \
  tests/test_gpu_ddp.py tests/test_gpu_ctc_head.py -s > gpurun_out/r5a_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r5a_tests.log; [ $rc -eq 0 ] || exit $rc
if [ -n "$DRIFT" ]; then bash tools/drift_ab.sh r5a; fi
