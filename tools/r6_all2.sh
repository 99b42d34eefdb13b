#!/bin/bash
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${TAG:-r6h}
timeout -k 10 1000 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_ddp.py tests/test_gpu_parity_step.py -k "two_ranks or bf16_layers" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "FAILED|passed|failed" gpurun_out/${TAG}_tests.log | tail -12
case $rc in 124|134|137|139) exit $rc;; esac
TAG=$TAG bash tools/r6_pmc.sh
