#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats kernel_stats.csv as a markdown table.
usage: tools/prof_summary.py run_kernel_stats.csv [steps]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else None
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("| share | calls | avg us | min us | total ms | kernel |")
print("|---:|---:|---:|---:|---:|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    name = r["Name"].replace("|", "/")
    if len(name) > 100:
        name = name[:100] + "..."
    print(f"| {float(r['TotalDurationNs']) / tot * 100:.1f}% | {r['Calls']} | "
          f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
          f"{float(r['TotalDurationNs']) / 1e6:.2f} | `{name}` |")
print(f"\ntotal GPU kernel time {tot / 1e6:.2f} ms" + (f" over {steps} steps = {tot / 1e6 / steps:.2f} ms/step" if steps else ""))
