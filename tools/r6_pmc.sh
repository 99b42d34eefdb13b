#!/bin/bash
# L2 hit / miss and fetch counters of the hand-written TN GEMM (tile_m 2) against the library's
# gate-forward kernel: one rocprofv3 --pmc pass per counter group, tools/tn_bench.py gate fwd.
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
TAG=${TAG:-r6h}
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d gpurun_out/pmc/${TAG}_p$i -o out --output-format csv -- \
    python3 tools/tn_bench.py --tm 2 --shapes 0 --nolib > gpurun_out/pmc/${TAG}_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/pmc/${TAG}_p$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/pmc/*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name", "")[:60], r.get("Counter_Name"))
        agg[k][0] += 1
        agg[k][1] += float(r.get("Counter_Value", 0))
    print(f)
    for (kn, cn), (n, v) in sorted(agg.items()):
        if "tnw32" in kn or "Cijk" in kn:
            print(f"  {kn:60s} {cn:32s} per-dispatch {v / n:.4g} (n={n})")
PY
