#!/bin/bash
# The CTC A/B (tools/r5_ctc.sh) and then the whole GPU test suite, one test process.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5z}
bash tools/r5_ctc.sh || exit $?
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_gpu_tests.log; exit $rc
