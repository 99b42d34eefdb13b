set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in xlstm rnnt; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof_$w" -o run -- \
  python3 "$R/bench.py" --workload $w --steps 2 --warmup 2 --cpu-baseline off > "$O/bench_prof_$w.json" 2> "$O/bench_prof_$w.err"
python3 "$R/tools/trace_tail.py" "$O/prof_$w/run_kernel_trace.csv" 4 2 "lucy_scan|joint_|mlstm_" \
  > "$O/prof_$w/trace_tail.md" || echo "trace_tail failed"
find "$O/prof_$w" -type f ! -name "*kernel_stats.csv" ! -name "trace_tail.md" -delete
done
echo done
