#!/bin/bash
# Graph-replayed segments: the bitwise test, then bench eager vs graph on one box (+ host probe),
# then the MFMA-busy PMC pass over the GEMM / scan kernels.  Every GPU step under its own limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5h}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_graphs.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/${TAG}_graph_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_graph_tests.log; [ $rc -eq 0 ] || exit $rc
for mode in off on off on; do
  timeout -k 10 300 python3 -X faulthandler -u bench.py --steps 20 --warmup 5 --cpu-baseline off --graph $mode \
    >> gpurun_out/${TAG}_graph_bench.jsonl 2>> gpurun_out/${TAG}_graph_bench.err || exit $?
done
timeout -k 10 300 python3 -X faulthandler -u bench.py --steps 4 --warmup 5 --cpu-baseline off --graph on \
  --host-probe > gpurun_out/${TAG}_graph_probe.log 2>&1 || exit $?
grep -h "host issue" gpurun_out/${TAG}_graph_probe.log
python3 - <<EOF
import json
for l in open("gpurun_out/${TAG}_graph_bench.jsonl"):
    d = json.loads(l)
    print(d["launch"][:9], d["value"], d["ms_per_step"], d["roofline"]["frac"])
EOF
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  GRBM_GUI_ACTIVE -f csv --kernel-include-regex "wgrad_kernel|tn256|scan_bwd|Cijk" \
  -d "$R/gpurun_out/${TAG}_pmc_mfma" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 \
  --cpu-baseline off > "$R/gpurun_out/${TAG}_pmc_mfma.log" 2>&1
rc=$?
find "$R/gpurun_out/${TAG}_pmc_mfma" -type f ! -name "*counter_collection.csv" -delete
exit $rc
