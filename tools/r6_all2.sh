#!/bin/bash
# Round-6: the whole GPU suite (new DDP / parity / LN-fold tests included), then the default
# bench line.  Each step has its own limit.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
TAG=${TAG:-r6h}
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_gpu_tests.log | head -20
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc2=$?; echo "bench rc=$rc2"; cat gpurun_out/${TAG}_bench.json | cut -c1-600
exit $rc
