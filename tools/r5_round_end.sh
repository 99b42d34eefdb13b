#!/bin/bash
# Round-5 closing GPU run: the whole GPU test suite, then the measurement set
# (tools/r5_final_prof.sh), then the stream bench over K = 1, 2, 4, 8 frames per call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5f}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
TAG=$TAG bash tools/r5_final_prof.sh || exit $?
cd "$R"
timeout -k 10 300 python3 -u tools/stream_bench.py --frames 128 --batches 1,16,64 --engines frame \
  --dtypes bfloat16 --ks 1,2,4,8 --no-reference > gpurun_out/${TAG}_stream_k.jsonl 2> gpurun_out/${TAG}_stream_k.err
rc=$?; cat gpurun_out/${TAG}_stream_k.jsonl; exit $rc
