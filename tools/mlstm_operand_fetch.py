#!/usr/bin/env python3
"""mLSTM backward: fetched bytes per operand from the FETCH_SIZE differences of builds that skip
one operand's loads (SC_ML_ABL 4096 q, 8192 k, 16384 v, 32768 dh, 65536 h, 131072 state image;
tools/r6_mlpmc.sh), converted with tools/mlstm_traffic.py's calibration for that operand's read
pattern and set against the operand's algorithmic bytes (read once per role that reads it).

usage: tools/mlstm_operand_fetch.py gpurun_out   (reads mlpmc_<tag>_FETCH_SIZE/*counter_collection.csv)
"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mlstm_traffic import CAL, QK, ST, VV  # noqa: E402

# operand: (ablation tag, algorithmic HBM bytes per launch, pattern).  Both roles read q, k, v,
# dh and h; the design counts them once (the second role of a sequence runs on the same XCD and
# should find the rows in its L2), so a ratio near 2 names an operand both roles fetch from HBM.
OPS = {
    "q": ("ml4096", QK, "seg192"),
    "k": ("ml8192", QK, "seg192"),
    "v": ("ml16384", VV, "seg384"),
    "dh": ("ml32768", VV, "stream"),
    "h": ("ml65536", VV, "stream"),
    "state image": ("ml131072", ST, "stream"),
}


def fetch_per_launch(d, tag):
    paths = glob.glob(os.path.join(d, f"mlpmc_{tag}_FETCH_SIZE", "**", "*counter_collection.csv"),
                      recursive=True)
    vals = [float(r["Counter_Value"]) * 1024.0 for p in paths for r in csv.DictReader(open(p))
            if r["Counter_Name"] == "FETCH_SIZE" and "mlstm_bw_walk" in r["Kernel_Name"]]
    if not vals:
        sys.exit(f"no mlstm_bw_walk FETCH_SIZE rows for {tag} under {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    base, n = fetch_per_launch(d, "base")
    print(f"baseline raw FETCH_SIZE per launch {base / 1e6:.1f} MB ({n} dispatches)")
    print("| operand | raw FETCH drop (MB) | calibrated bytes (MB) | algorithmic (MB) | ratio |")
    print("|---|---:|---:|---:|---:|")
    tot_c = tot_a = 0.0
    for name, (tag, alg, pat) in OPS.items():
        f, _ = fetch_per_launch(d, tag)
        drop = base - f
        cal = drop * CAL[pat]
        tot_c += cal
        tot_a += alg
        print(f"| {name} | {drop / 1e6:.1f} | {cal / 1e6:.1f} | {alg / 1e6:.1f} | {cal / alg:.2f} |")
    print(f"| all six | | {tot_c / 1e6:.1f} | {tot_a / 1e6:.1f} | {tot_c / tot_a:.2f} |")


if __name__ == "__main__":
    main()
