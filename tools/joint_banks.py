#!/usr/bin/env python3
"""LDS bank-conflict count of the joint kernels' image accesses (csrc/rnnt.hip wimg / pimg_off),
by the gfx950 banking rules of MI355X_MICROARCH.md §LDS: per lane group, extra cycles = (max
distinct addresses on one bank) - 1.  usage: python tools/joint_banks.py"""


def wswz(row):
    return (((row >> 1) & 1) << 2) | ((row >> 2) & 3)


def wimg(row, chunk):
    return row * 128 + 16 * (chunk ^ wswz(row))


def pimg_off(row, col):
    return wimg(row, col >> 3) + 8 * (((col >> 2) & 1) ^ (row & 1))


B128_GROUPS = [[*range(0, 4), *range(12, 16), *range(20, 28)],
               [*range(4, 12), *range(16, 20), *range(28, 32)]]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]
HALVES = [list(range(32)), list(range(32, 64))]
W64_GROUPS = [list(range(16 * i, 16 * i + 16)) for i in range(4)]


def extra(groups, addr, nbytes, mod):
    tot = 0
    for grp in groups:
        banks = {}
        for l in grp:
            a = addr(l)
            for d in range(nbytes // 4):
                banks.setdefault((a // 4 + d) % mod, set()).add(a + 4 * d)
        tot += max(len(v) for v in banks.values()) - 1
    return tot


def tr(R0, C0, off):
    def addr(lane):
        i = lane & 15
        q, p = i >> 2, i & 3
        h, g1 = lane >> 5, (lane >> 4) & 1
        return off(R0(h) + q, C0(g1) + 4 * p)
    return addr


def main():
    plain = lambda row, col: wimg(row, col >> 3) + 8 * ((col >> 2) & 1)
    cases = {}
    for s in range(4):   # W / z row reads (logits A and B operands)
        cases[f"b128 row read s={s}"] = extra(B128_GROUPS, lambda l: wimg(l & 31, 2 * s + (l >> 5)), 16, 64)
    for s2 in range(2):
        for jb in range(2):
            for k8 in (0, 8):
                cases[f"tr z/W s2={s2} jb={jb} +{k8}"] = extra(
                    HALVES, tr(lambda h: 16 * s2 + k8 + 4 * h, lambda g1: jb * 32 + 16 * g1, plain), 8, 64)
        for k8 in (0, 8):
            cases[f"tr p s2={s2} +{k8}"] = extra(
                HALVES, tr(lambda h: 16 * s2 + k8 + 4 * h, lambda g1: 16 * g1, pimg_off), 8, 64)
    for g in range(4):
        cases[f"p write g={g}"] = extra(W64_GROUPS, lambda l: pimg_off(l & 31, 8 * g + 4 * (l >> 5)), 8, 32)
    bad = {k: v for k, v in cases.items() if v}
    for k, v in cases.items():
        print(f"{k:28s} extra cycles {v}")
    print("conflict-free" if not bad else f"CONFLICTS: {bad}")
    return 1 if bad else 0


if __name__ == "__main__":
    raise SystemExit(main())
