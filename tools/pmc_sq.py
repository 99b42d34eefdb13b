"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one row per dispatch and
counter), e.g. the SQ wait breakdown of the mLSTM kernels:

  rocprofv3 --pmc SQ_WAVE_CYCLES,SQ_WAIT_ANY,... --output-format csv -d gpurun_out/p -- python3 ...
  python tools/pmc_sq.py gpurun_out/p [substring]

Prints, per kernel (template arguments kept), the mean of every counter over its dispatches and,
when the SQ cycle counters are present, the wave-cycle split WAIT_ANY / WAIT_INST_ANY /
ACTIVE_INST_ANY (disjoint; MI355X_MICROARCH.md "rocprofv3 PMC slots")."""
import collections
import csv
import glob
import os
import sys


def load(d, sub=""):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("sc::(anonymous namespace)::", "").rsplit("(", 1)[0]
            if sub and sub not in k:
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for k, c in sorted(load(d, sub).items()):
        print(k)
        for n in sorted(c):
            print(f"  {n:24s} {c[n]:16.0f}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            parts = [(n, c[n] / wc) for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")
                     if n in c]
            print("  split " + "  ".join(f"{n[3:]}={f:.3f}" for n, f in parts))


if __name__ == "__main__":
    main()
