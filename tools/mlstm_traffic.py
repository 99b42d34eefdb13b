#!/usr/bin/env python3
"""mLSTM HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes, converted to bytes
with the access-pattern calibration of tools/fetch_probe.hip instead of one x2 factor.

FETCH_SIZE counts a 16-byte-per-lane streaming read at half its bytes (x2.000, the guide's gfx950
rule), but the walks read q / k / v as row SEGMENTS of the xLSTM's fused projection (192 B of q or
k, 384 B of v, 128 B of one v column block, at a 4,624-B row stride), which the probe measured at
x1.263, x1.548 and x1.067.  Each kernel's raw counter is converted with the harmonic blend of its
operands' factors weighted by their algorithmic bytes (so the conversion is exact when the kernel
reads each operand once; an operand read twice from HBM shows up as traffic above 1.0x).

usage: tools/mlstm_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv
"""
import collections
import csv
import re
import sys

# C4 bench cell: B = 32, NH = 4 (BH = 128), T = 1536, DQ = 96, DV = 192, bf16 operands
BH, T, DQ, DV, NC = 128, 1536, 96, 192, 1536 // 64
E = 2
QK = BH * T * DQ * E          # one of q / k
VV = BH * T * DV * E          # v, h, dh
ST = BH * NC * DQ * DV * E    # chunk state image
CAL = {"stream": 2.000, "seg192": 1.263, "seg384": 1.548, "seg128": 1.067}
WCAL = {"stream": 1.000, "seg192": 0.923, "tile": 0.848}
# (operand, bytes, read pattern) per kernel, and the writes
READS = {
    "mlstm_fw_walk": [("k", QK, "seg192"), ("v column block", VV, "seg128")],
    "mlstm_fw_out": [("q", QK, "seg192"), ("k", QK, "seg192"), ("v", VV, "seg384"),
                     ("state image", ST, "stream")],
    "mlstm_bw_walk": [("q", QK, "seg192"), ("k", QK, "seg192"), ("v", VV, "seg384"),
                      ("h", VV, "stream"), ("dh", VV, "stream"), ("state image", ST, "stream")],
}
WRITES = {
    "mlstm_fw_walk": [("state image", ST, "stream")],
    "mlstm_fw_out": [("h", VV, "stream")],
    "mlstm_bw_walk": [("dq", QK, "seg192"), ("dk", QK, "seg192"), ("dv", VV, "tile")],
}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        m = re.search(r"(mlstm_(fw_walk|fw_out|bw_walk))", r["Kernel_Name"])
        if m:
            acc[m.group(1)].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def blend(ops, table):
    tot = sum(b for _, b, _ in ops)
    return tot / sum(b / table[p] for _, b, p in ops), tot


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    print("| kernel | FETCH_SIZE raw | factor | reads (calibrated) | reads (algorithmic) | "
          "WRITE_SIZE raw | factor | writes | writes (algorithmic) | total / algorithmic |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in ("mlstm_fw_walk", "mlstm_fw_out", "mlstm_bw_walk"):
        fr, fa = blend(READS[k], CAL)
        wr, wa = blend(WRITES[k], WCAL)
        rd, wt = fetch.get(k, 0.0) * fr, write.get(k, 0.0) * wr
        print(f"| {k} | {fetch.get(k, 0) / 1e6:.1f} MB | x{fr:.3f} | {rd / 1e6:.1f} MB | {fa / 1e6:.1f} MB "
              f"| {write.get(k, 0) / 1e6:.1f} MB | x{wr:.3f} | {wt / 1e6:.1f} MB | {wa / 1e6:.1f} MB "
              f"| {(rd + wt) / (fa + wa):.2f} |")


if __name__ == "__main__":
    main()
