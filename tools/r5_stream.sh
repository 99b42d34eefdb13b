#!/bin/bash
# Round-5 streaming run: the streaming GPU tests, then tools/stream_bench.py (frame engine,
# wavefront vs frame-by-frame schedule, fp32 and bf16, 1-256 streams).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5s}
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_streaming.py \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u tools/stream_bench.py --frames 128 --batches ${BATCHES:-1,16,64,256} --engines frame --ks ${KS:-1,8} \
  --dtypes float32,bfloat16 --no-reference > gpurun_out/${TAG}_stream.jsonl 2> gpurun_out/${TAG}_stream.err
rc=$?; cat gpurun_out/${TAG}_stream.jsonl; exit $rc
