#!/usr/bin/env python3
"""Per-launch HBM traffic of the scan and mLSTM kernels from two rocprofv3 PMC passes.

usage: tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv [out.json KEY]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports half the bytes of
a 16-byte-per-lane streaming read (MI355X_MICROARCH.md, HBM section); the scans read every gate
byte with 16-byte LDS-DMA pieces, so fetch bytes = 2 x FETCH_SIZE x 1024.  WRITE_SIZE is taken
as is (calibrated on the scan forward: its 52 MB of bf16 output + checkpoint read back exactly).
Prints JSON {bench_kernel_name: {"hbm_bytes_per_launch", "fetch_bytes", "write_bytes",
"dispatches"}} keyed like bench.py's "kernels" entries; with out.json, merges it into that table
under KEY = "<workload>/<dtype>" of the profiled bench run (e.g. "ctc/bf16"), which is what
bench.py's roofline.traffic looks up (no entry for the run's workload and dtype: null).
"""
import csv
import json
import sys
from collections import defaultdict

NAMES = {"lucy_scan_fwd_kernel": "lucy_scan_fwd", "lucy_scan_bwd_kernel": "lucy_scan_bwd",
         "decay_scan_fwd_kernel": "decay_scan_fwd", "decay_scan_bwd_kernel": "decay_scan_bwd",
         # the mLSTM walks read q / k / v / h / dh and the state image as 16-byte-per-lane rows
         # (the same FETCH_SIZE calibration)
         # a forward is the state walk plus the chunk-parallel output kernel: their per-dispatch
         # averages add up to one launch of sc_mlstm_fwd
         "mlstm_fw_walk": "mlstm_fwd", "mlstm_fw_out": "mlstm_fwd", "mlstm_bw_walk": "mlstm_bwd"}


def per_kernel(path, counter):
    """{name: (bytes per launch = sum over the name's kernels of their per-dispatch means,
    dispatches of its first kernel)}"""
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for frag, name in NAMES.items():
            if frag in r["Kernel_Name"]:
                acc[name][frag].append(float(r["Counter_Value"]) * 1024.0)
    return {name: (sum(sum(v) / len(v) for v in frags.values()), len(next(iter(frags.values()))))
            for name, frags in acc.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for name in sorted(set(fetch) & set(write)):
        f = 2.0 * fetch[name][0]
        w = write[name][0]
        out[name] = {"hbm_bytes_per_launch": round(f + w), "fetch_bytes": round(f),
                     "write_bytes": round(w), "dispatches": fetch[name][1]}
    if len(sys.argv) > 3:
        key = sys.argv[4]
        if "/" not in key:
            sys.exit("KEY must be <workload>/<dtype>, e.g. ctc/bf16")
        try:
            prev = json.load(open(sys.argv[3]))
        except (OSError, ValueError):
            prev = {}
        prev.setdefault(key, {}).update(out)
        out = prev
    txt = json.dumps(out, indent=1)
    if len(sys.argv) > 3:
        open(sys.argv[3], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
