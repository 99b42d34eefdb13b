#!/bin/bash
# Full round measurement on one GPU box: GPU tests, the three bench workloads, and the
# rocprofv3 kernel trace + PMC passes of the default (C2) bench.  usage: tools/round_run.sh TAG
# Every GPU step has its own time limit and the steps are chained (set -e): after a failure
# nothing else touches the GPU.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r2}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
if [ -z "$SKIP_TESTS" ]; then
  echo "gpu tests"
  timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$O/gputest_$TAG.log" 2>&1 || { tail -30 "$O/gputest_$TAG.log"; exit 1; }
  tail -3 "$O/gputest_$TAG.log"
fi
for w in rnnt xlstm; do
  echo "bench $w"
  timeout -k 10 300 python3 "$R/bench.py" --workload $w --steps 8 --warmup 4 \
    > "$O/bench_${w}_$TAG.json" 2> "$O/bench_${w}_$TAG.err" || { tail -30 "$O/bench_${w}_$TAG.err"; exit 1; }
  cat "$O/bench_${w}_$TAG.json"
done
bash "$R/tools/gpu_profile.sh" "$TAG"
cat "$O/bench_$TAG.json"
