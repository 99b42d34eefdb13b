#!/bin/bash
# Graph replay vs eager for the C5 (rnnt) and C4 (xlstm) workloads, one box, plus smoke().
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
TAG=${TAG:-r5j}
for wl in rnnt xlstm; do
  for mode in off on; do
    timeout -k 10 400 python3 -X faulthandler -u bench.py --workload $wl --steps 10 --warmup 3 \
      --cpu-baseline off --graph $mode >> gpurun_out/${TAG}_graph_wl.jsonl \
      2>> gpurun_out/${TAG}_graph_wl.err || exit $?
  done
done
python3 - <<PY
import json
for l in open("gpurun_out/${TAG}_graph_wl.jsonl"):
    d = json.loads(l)
    print(d["config"]["workload"][:30], d["launch"][:9], d["value"], d["ms_per_step"], d["loss_last"])
PY
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_smoke.log; exit $rc
