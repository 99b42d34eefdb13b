#!/bin/bash
# Round-6 closing GPU run: the whole GPU test suite, smoke(), the default bench line (with the
# CPU baseline), the kernel-trace / PMC profile (tools/gpu_profile.sh, bench skipped) and the
# C4 / C5 lines.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r6z}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 500 python3 -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || exit 1
tail -c 600 gpurun_out/bench_${TAG}.json
SKIP_BENCH=1 bash tools/gpu_profile.sh $TAG || exit 1
cd "$R"
for wl in rnnt xlstm; do
  timeout -k 10 300 python3 -u bench.py --workload $wl --cpu-baseline off > gpurun_out/bench_${TAG}_$wl.json \
    2> gpurun_out/bench_${TAG}_$wl.err || exit 1
done
echo done
