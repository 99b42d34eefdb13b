#!/bin/bash
# One round's measurement on the GPU box: the default bench line, a rocprofv3 kernel-trace/stats
# profile of a short bench, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE; never combined
# with other traces) over the scan kernels.  usage: tools/gpu_profile.sh TAG
# Outputs under gpurun_out/: bench_TAG.json, prof_TAG/, pmc_{fetch,write}_TAG/.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r1}
O=$R/gpurun_out
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
if [ -z "$SKIP_BENCH" ]; then
  echo "bench"
  timeout -k 10 500 python3 "$R/bench.py" > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err"
fi
echo "kernel trace"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 --cpu-baseline off > "$O/bench_prof_$TAG.json" 2> "$O/bench_prof_$TAG.err"
echo "pmc fetch"
timeout -k 10 500 rocprofv3 --pmc FETCH_SIZE -f csv --kernel-include-regex "scan" -d "$O/pmc_fetch_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-baseline off > "$O/pmc_fetch_$TAG.log" 2>&1
echo "pmc write"
timeout -k 10 500 rocprofv3 --pmc WRITE_SIZE -f csv --kernel-include-regex "scan" -d "$O/pmc_write_$TAG" -o run -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-baseline off > "$O/pmc_write_$TAG.log" 2>&1
# the timed steps' dispatches of the hot kernels (bench --steps 5 --warmup 2, events in the last 2)
python3 "$R/tools/trace_tail.py" "$O/prof_$TAG/run_kernel_trace.csv" 7 2 "lucy_scan|joint_|mlstm_" \
  "$O/prof_$TAG/hot_dispatches.csv" > "$O/prof_$TAG/trace_tail.md" || echo "trace_tail failed"
# keep only the summaries (gpurun copies back at most 64 MiB)
find "$O/prof_$TAG" "$O/pmc_fetch_$TAG" "$O/pmc_write_$TAG" -type f \
  ! -name "*kernel_stats.csv" ! -name "*counter_collection.csv" ! -name "hot_dispatches.csv" \
  ! -name "trace_tail.md" -delete
du -sh "$O"
echo done
