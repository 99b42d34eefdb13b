#!/usr/bin/env python3
"""Per-kernel launch durations from a rocprofv3 --kernel-trace CSV, restricted to the dispatches
of the bench's timed steps, so that the profile's average and bench.py's HIP-event average cover
the same launches.

usage: tools/trace_tail.py run_kernel_trace.csv TOTAL_STEPS TIMED_STEPS [regex] [out.csv]
  The last TIMED_STEPS / TOTAL_STEPS of each kernel's dispatches (in start order) are the timed
  ones (bench.py records its HIP events in its last --timing-steps steps).  Prints avg / min /
  max per kernel over all dispatches and over the timed ones; out.csv keeps the matching
  kernels' per-dispatch durations (name, start order, ns)."""
import csv
import re
import sys
from collections import defaultdict


def main():
    path, total, timed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    pat = re.compile(sys.argv[4] if len(sys.argv) > 4 else "lucy_scan|joint_|mlstm_")
    out = sys.argv[5] if len(sys.argv) > 5 else None
    runs = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not pat.search(name):
            continue
        runs[name].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows = []
    print("| kernel | dispatches | avg us (all) | timed dispatches | avg us (timed) | min | max |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for name, v in sorted(runs.items()):
        v.sort()
        d = [x[1] for x in v]
        n_t = max(1, round(len(d) * timed / total))
        t = d[-n_t:]
        short = name if len(name) < 70 else name[:70] + "..."
        print(f"| `{short}` | {len(d)} | {sum(d) / len(d) / 1e3:.1f} | {n_t} | "
              f"{sum(t) / len(t) / 1e3:.1f} | {min(t) / 1e3:.1f} | {max(t) / 1e3:.1f} |")
        rows += [(name, i, x) for i, x in enumerate(d)]
    if out:
        with open(out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "dispatch", "duration_ns"])
            w.writerows(rows)


if __name__ == "__main__":
    main()
