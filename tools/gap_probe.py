"""Idle gaps between kernels in a rocprofv3 kernel trace (which part of the step is dispatch
overhead rather than kernel time).  usage: tools/gap_probe.py run_kernel_trace.csv [last_n_kernels]

Prints the span, the summed kernel time and the gap histogram over the last N dispatches."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if last:
        ev = ev[-last:]
    span = ev[-1][1] - ev[0][0]
    busy = sum(e - s for s, e, _ in ev)
    gaps = []
    for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
        gaps.append((s1 - e0, n0[:60], n1[:60]))
    pos = [g for g, _, _ in gaps if g > 0]
    print(f"dispatches {len(ev)}  span {span / 1e3:.1f} us  kernel sum {busy / 1e3:.1f} us  "
          f"idle {(span - busy) / 1e3:.1f} us ({100 * (span - busy) / span:.1f}%)")
    if pos:
        pos.sort()
        print(f"gaps>0: n={len(pos)} median {pos[len(pos) // 2] / 1e3:.2f} us  "
              f"p90 {pos[int(len(pos) * 0.9)] / 1e3:.2f} us  max {pos[-1] / 1e3:.2f} us")
    gaps.sort(reverse=True)
    for g, a, b in gaps[:12]:
        print(f"  {g / 1e3:8.2f} us  after {a}  before {b}")


if __name__ == "__main__":
    main()
