#!/usr/bin/env python3
"""Bytes per counter unit for each tools/fetch_probe.hip pattern.

usage: tools/fetch_probe.py PROBE_STDOUT FETCH_counter_collection.csv WRITE_counter_collection.csv
Prints, per kernel, the known byte count, FETCH_SIZE / WRITE_SIZE of its last dispatch (KiB x
1024) and the factor known / counter -- the multiplier that turns the counter into bytes for that
access pattern."""
import csv
import sys


def last_by_kernel(path, counter):
    out = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out[r["Kernel_Name"]] = float(r["Counter_Value"]) * 1024.0   # later dispatches win
    return out


def main():
    known = {}
    for line in open(sys.argv[1]):
        name, _, n = line.strip().rpartition(" ")
        if name and n.isdigit():
            known[name] = int(n)
    fetch = last_by_kernel(sys.argv[2], "FETCH_SIZE")
    write = last_by_kernel(sys.argv[3], "WRITE_SIZE")
    print("| pattern | bytes moved | FETCH_SIZE bytes | WRITE_SIZE bytes | bytes per counter byte |")
    print("|---|---:|---:|---:|---:|")
    def norm(k):   # "void rd_seg<192, 0>(char const*, ...)" -> "rd_seg<192,0>"
        k = k.split("(")[0].replace(" ", "")
        return k[4:] if k.startswith("void") else k
    fetch = {norm(k): v for k, v in fetch.items()}
    write = {norm(k): v for k, v in write.items()}
    for name, n in known.items():
        key = norm(name)
        f, w = fetch.get(key, 0.0), write.get(key, 0.0)
        c = f if name.startswith("rd") else w
        print(f"| {name} | {n} | {f:.0f} | {w:.0f} | {n / c if c else float('nan'):.3f} |")


if __name__ == "__main__":
    main()
