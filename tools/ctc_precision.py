"""CTC lattice precision study (tool, not product): numpy emulation of ctc_ab's fp32 arithmetic.

Emulates the HIP lattice's number formats -- base-2 log space, fp32 state values, re-centring on
the lattice max every R steps with an fp64 running offset -- and variants of it, against the fp64
oracle (oracle/ctc.py), to find which rounding dominates the dlogits error at T=1500, U=150.

    python tools/ctc_precision.py [--T 1500] [--U 150] [--scale 1.0]

Variants:
  cur      the shipped kernel: re-centre every 48 steps
  every    re-centre every step (the best a plain fp32 log-space lattice can do)
  cshift   subtract a per-step uniform c_t = max_s e_t(s) from the emissions (fp64 sum of c_t)
  cshift16 cshift + re-centre every 16 steps
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import ctc as octc  # noqa: E402

F = np.float32
LOG2E = F(1.4426950408889634)
DEAD = F(-1e30)


def lse3(a, b, c):
    m = np.maximum(np.maximum(a, b), c)
    md = np.median(np.stack([a, b, c]), axis=0).astype(F)
    lo = np.minimum(np.minimum(a, b), c)
    s = F(1) + np.exp2(md - m) + np.exp2(lo - m)
    return (m + np.log2(s).astype(F)).astype(F)


def lattice(e2, skip, R, beta=False):
    """e2: (T, S) fp32 base-2 emissions (dead = -1e30), returns values (T,S) fp32 and fp64 offs (T,)"""
    T, S = e2.shape
    v = np.full(S, DEAD, F)
    out = np.empty((T, S), F)
    offs = np.zeros(T)
    off = 0.0
    for i in range(T):
        if i == 0:
            if beta:
                v[S - 1] = e2[0, S - 1]
                if S > 1:
                    v[S - 2] = e2[0, S - 2]
            else:
                v[0] = e2[0, 0]
                if S > 1:
                    v[1] = e2[0, 1]
        else:
            if beta:
                n1 = np.concatenate([v[1:], [DEAD]]).astype(F)
                n2 = np.concatenate([v[2:], [DEAD, DEAD]]).astype(F)
                n2 = np.where(skip, n2, DEAD).astype(F)
            else:
                n1 = np.concatenate([[DEAD], v[:-1]]).astype(F)
                n2 = np.concatenate([[DEAD, DEAD], v[:-2]]).astype(F)
                n2 = np.where(skip, n2, DEAD).astype(F)
            v = (lse3(v, n1, n2) + e2[i]).astype(F)
            v = np.maximum(v, DEAD)
        if R and (i + 1) % R == 0:
            m = v.max()
            v = (v - m).astype(F)
            off += float(m)
        out[i] = v
        offs[i] = off
    return out, offs


def hip_like(x, tgt, R, cshift=False):
    """x (T,V) fp32 logits -> dlogits fp64 (T,V) via the emulated fp32 lattice"""
    T, V = x.shape
    U = len(tgt)
    S = 2 * U + 1
    ext = np.zeros(S, np.int64)
    ext[1::2] = tgt
    m = x.max(1, keepdims=True)
    lse = (m + np.log(np.exp(x - m).sum(1, keepdims=True, dtype=F))).astype(F)
    lp2 = ((x - lse) * LOG2E).astype(F)          # base-2 log-probs as the emit kernel rounds them
    e2 = lp2[:, ext]
    c = np.zeros(T)
    if cshift:
        c = e2.max(1).astype(np.float64)
        e2 = (e2 - c[:, None].astype(F)).astype(F)
    skip = np.zeros(S, bool)
    skip[2:] = (ext[2:] != 0) & (ext[2:] != ext[:-2])
    skip_b = np.zeros(S, bool)
    skip_b[:-2] = skip[2:]
    al, oa = lattice(e2, skip, R)
    be, ob = lattice(e2[::-1], skip_b, R, beta=True)
    be, ob = be[::-1], ob[::-1]
    ca = np.cumsum(c)                      # alpha_t holds sum_{t'<=t} c
    cb = np.cumsum(c[::-1])[::-1]          # beta_t holds sum_{t'>=t} c
    # alpha's offset at t is the one in force after step t; beta's likewise
    ll2 = np.logaddexp2(al[-1, -1].astype(np.float64), al[-1, -2].astype(np.float64)) + oa[-1] + ca[-1]
    ab = al.astype(np.float64) + be.astype(np.float64)     # fp32 sum in the kernel: round it
    ab = (al + be).astype(F).astype(np.float64)
    koff = oa + ob + ca + cb - ll2                       # fp64 offsets folded (kernel: one float)
    koff = koff.astype(F).astype(np.float64)
    lcab = np.full((T, V), -np.inf)
    for s in range(S):
        lcab[:, ext[s]] = np.logaddexp2(lcab[:, ext[s]], ab[:, s])
    lpn = lp2.astype(np.float64)
    g = np.exp2(lpn) - np.exp2(lcab + koff[:, None] - lpn)
    return -ll2 / LOG2E, g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=1500)
    ap.add_argument("--U", type=int, default=150)
    ap.add_argument("--V", type=int, default=1024)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--real", action="store_true",
                    help="the logits of tests/test_gpu_parity_step.py's C2 fp32 step (oracle forward)")
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    x = (rng.standard_normal((a.T, a.V)) * a.scale).astype(F)
    tgt = rng.integers(1, a.V, a.U)
    if a.real:
        from oracle import lucy_step
        from tests.test_gpu_parity_step import oracle_params, step_inputs
        feats, tok, U = step_inputs(2, a.T, 5)
        logits = lucy_step.forward(oracle_params(), feats, 6, 512)[0]
        x = np.ascontiguousarray(logits[a.seed]).astype(F)
        tgt = tok[a.seed, :U[a.seed]]
        print(f"real logits row {a.seed}: std {x.std():.3f}, max {x.max():.2f}, U {len(tgt)}")
    nll64, g64 = octc.ctc_single(octc.log_softmax(x.astype(np.float64)), tgt)
    print(f"T={a.T} U={a.U} scale={a.scale}: nll64 {nll64:.6f}")
    for name, R, cs in (("cur", 48, False), ("every", 1, False), ("cshift", 48, True),
                        ("cshift16", 16, True)):
        nll, g = hip_like(x, tgt, R, cs)
        e = np.linalg.norm(g - g64) / np.linalg.norm(g64)
        print(f"  {name:9s} nll {nll:.6f} (rel {abs(nll - nll64) / nll64:.1e})  dlogits rel {e:.2e}")


if __name__ == "__main__" and "--rnnt" not in sys.argv:
    main()


# ------------------------------------------------------------------------------------ RNN-T ----
def rnnt_lattice32(lb2, ly2, R):
    """fp32 emulation of rnnt_ab (base 2, re-centre every R diagonals): returns the alpha and
    beta node values (fp64 after adding their fp64 offsets) and log2 P."""
    T, U1 = lb2.shape
    U = U1 - 1
    nd = T + U
    A = np.full((T, U1), -np.inf)
    Bt = np.full((T, U1), -np.inf)
    v = np.full(U1, DEAD, F)        # lane u holds node (n - u, u)
    off = 0.0
    uu = np.arange(U1)
    for n in range(nd):
        t = n - uu
        ok = (t >= 0) & (t < T)
        if n == 0:
            nv = np.where(uu == 0, F(0), DEAD).astype(F)
        else:
            tp = np.clip(t - 1, 0, T - 1)
            c1 = np.where((t >= 1) & ok, (v + lb2[tp, uu]).astype(F), DEAD)
            vn = np.concatenate([[DEAD], v[:-1]]).astype(F)
            tc = np.clip(t, 0, T - 1)
            c2 = np.where((uu >= 1) & ok, (vn + ly2[tc, np.maximum(uu - 1, 0)]).astype(F), DEAD)
            m = np.maximum(c1, c2)
            nv = (m + np.log2(np.exp2(c1 - m) + np.exp2(c2 - m)).astype(F)).astype(F)
        v = np.where(ok, np.maximum(nv, DEAD), DEAD).astype(F)
        if R and (n + 1) % R == 0:
            mx = v.max()
            if mx > DEAD / 2:
                v = (v - mx).astype(F)
                off += float(mx)
        A[t[ok], uu[ok]] = v[ok].astype(np.float64) + off
    logp = A[T - 1, U] + float(lb2[T - 1, U])
    v = np.full(U1, DEAD, F)
    off = 0.0
    for i in range(nd):
        n = nd - 1 - i
        t = n - uu
        ok = (t >= 0) & (t < T)
        if i == 0:
            nv = np.where(uu == U, lb2[T - 1, U], DEAD).astype(F)
        else:
            tc = np.clip(t, 0, T - 1)
            c1 = np.where((t + 1 < T) & ok, (v + lb2[tc, uu]).astype(F), DEAD)
            vn = np.concatenate([v[1:], [DEAD]]).astype(F)
            c2 = np.where((uu < U) & ok, (vn + ly2[tc, np.minimum(uu, U - 1)]).astype(F), DEAD)
            m = np.maximum(c1, c2)
            nv = (m + np.log2(np.exp2(c1 - m) + np.exp2(c2 - m)).astype(F)).astype(F)
        v = np.where(ok, np.maximum(nv, DEAD), DEAD).astype(F)
        if R and (i + 1) % R == 0:
            mx = v.max()
            if mx > DEAD / 2:
                v = (v - mx).astype(F)
                off += float(mx)
        Bt[t[ok], uu[ok]] = v[ok].astype(np.float64) + off
    return A, Bt, logp


def rnnt_grads2(A, Bt, lb2, ly2, logp):
    T, U1 = lb2.shape
    U = U1 - 1
    gb = np.zeros((T, U1))
    gb[:T - 1] = -np.exp2(A[:T - 1] + lb2[:T - 1] + Bt[1:] - logp)
    gb[T - 1, U] = -np.exp2(A[T - 1, U] + lb2[T - 1, U] - logp)
    gy = -np.exp2(A[:, :U] + ly2 + Bt[:, 1:] - logp)
    return gb, gy


def rnnt_study(R=32):
    """The C5 test's first sequence (tests/test_gpu_c5.py setup): blank / label log-probs from the
    fp64 joint, rounded to fp32 base 2 as rnnt_emit stores them."""
    import torch
    from oracle import lucy_step
    from tests.test_gpu_c5 import JKEYS  # noqa: F401
    from tests.test_gpu_parity_step import oracle_params
    rng = np.random.default_rng(21)
    T, U, V = 1500, 150, 1024
    feats = rng.standard_normal((2, T, 80)).astype(np.float32)
    tok = rng.integers(1, V, (2, U))
    p = oracle_params()
    logits = lucy_step.forward(p, feats, 6, 512)[0][0].astype(np.float64)
    g = torch.Generator().manual_seed(5)
    We = torch.randn(64, V, generator=g, dtype=torch.float64) * (4.0 / np.sqrt(V))
    Wp = torch.randn(64, 64, generator=g, dtype=torch.float64) / 8
    Wj = torch.randn(V, 64, generator=g, dtype=torch.float64) * (3.0 / 8)
    emb = torch.randn(V, 64, generator=g, dtype=torch.float64)
    prefix = torch.as_tensor(np.concatenate([[0], tok[0]]))
    enc_p = torch.as_tensor(logits) @ We.T
    pred_p = emb[prefix] @ Wp.T
    lb = np.empty((T, U + 1))
    ly = np.empty((T, U))
    y = torch.as_tensor(tok[0])
    for t0 in range(0, T, 100):
        z = torch.tanh(enc_p[t0:t0 + 100, None, :] + pred_p[None, :, :])
        lg = z @ Wj.T
        lp = lg - torch.logsumexp(lg, -1, keepdim=True)
        lb[t0:t0 + 100] = lp[..., 0].numpy()
        ly[t0:t0 + 100] = lp[:, torch.arange(U), y].numpy()
    lb2 = (lb.astype(F) * LOG2E).astype(F)
    ly2 = (ly.astype(F) * LOG2E).astype(F)
    lb2d, ly2d = lb2.astype(np.float64), ly2.astype(np.float64)
    nll, gb64, gy64 = lucy_step.rnnt_lattice(lb2d / np.log2(np.e), ly2d / np.log2(np.e))
    ref = np.concatenate([gb64.ravel(), gy64.ravel()])
    print(f"RNN-T T={T} U={U}: nll64 {nll:.6f}; blank lp mean {lb.mean():.2f}, label lp mean {ly.mean():.2f}")
    for name, R_, shift in (("cur", R, False), ("every", 1, False), ("shift", R, True),
                            ("dshift", R, "d")):
        if shift == "d":   # one constant per anti-diagonal n = t + u for both arcs leaving it
            nd = T + U
            tt, uu = np.meshgrid(np.arange(T), np.arange(U + 1), indexing="ij")
            kb = np.full(nd, -np.inf)
            np.maximum.at(kb, (tt + uu).ravel(), lb2d.ravel())
            np.maximum.at(kb, (tt[:, :U] + uu[:, :U]).ravel(), ly2d.ravel())
            kb = kb.astype(F).astype(np.float64)
            A, Bt, lp = rnnt_lattice32((lb2d - kb[tt + uu]).astype(F),
                                       (ly2d - kb[tt[:, :U] + uu[:, :U]]).astype(F), R_)
            Kc = np.concatenate([[0], np.cumsum(kb)])
            A = A + Kc[tt + uu]
            Bt = Bt + (Kc[nd] - Kc[tt + uu])
            lp = lp + Kc[nd]
        elif shift:   # per-frame blank and per-position label constants (every path has one of each)
            cb = lb2d.max(1)
            cy = ly2d.max(0)
            A, Bt, lp = rnnt_lattice32((lb2d - cb[:, None]).astype(F), (ly2d - cy[None, :]).astype(F), R_)
            # alpha(t,u) holds sum_{t'<t} cb + sum_{u'<u} cy; beta(t,u) the rest from (t,u) on
            Cb = np.concatenate([[0], np.cumsum(cb)])
            Cy = np.concatenate([[0], np.cumsum(cy)])
            A = A + Cb[:T, None] + Cy[None, :U + 1]
            Bt = Bt + (Cb[T] - Cb[:T, None]) + (Cy[U] - Cy[None, :U + 1])
            lp = lp + Cb[T] + Cy[U]
        else:
            A, Bt, lp = rnnt_lattice32(lb2, ly2, R_)
        gb, gy = rnnt_grads2(A, Bt, lb2d, ly2d, lp)
        e = np.linalg.norm(np.concatenate([gb.ravel(), gy.ravel()]) - ref) / np.linalg.norm(ref)
        print(f"  {name:6s} nll {-lp / np.log2(np.e):.6f}  arc-gradient rel {e:.2e}")


if __name__ == "__main__" and "--rnnt" in sys.argv:
    rnnt_study()
