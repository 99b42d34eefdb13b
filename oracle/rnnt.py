"""RNN-T (transducer) loss restated in numpy — TEST INFRASTRUCTURE ONLY.

The reference computes the RNN-T loss with the third-party ``warp_rnnt`` package
(model.py:97-105 calls it with ``log_probs, labels, frames_lengths, labels_lengths, blank_id,
compact, gather=True``; train.py:38-42, :144).  warp_rnnt is not vendored in /root/reference,
not in requirements.txt and not installable offline: **parity unpinned** against
it.  This module restates its published algorithm (Graves 2012, the transducer lattice warp_rnnt
implements) and is pinned instead against a brute-force sum over every monotonic alignment
(``brute_force_nll``) on tiny lattices (tests/test_oracle_golden.py).

Lattice for one sequence: log_probs lp[t, u, v] for t < T, u <= U (U = label count);
  alpha[0,0] = 0
  alpha[t,u] = logaddexp(alpha[t-1,u] + lp[t-1,u,blank], alpha[t,u-1] + lp[t,u-1,y[u-1]])
  log P(y|x) = alpha[T-1,U] + lp[T-1,U,blank]
The loss is -log P.  Gradients are w.r.t. the gathered entries only (gather=True): the blank
and the next-label log-prob of every (t, u) node.
"""
import itertools

import numpy as np


def rnnt_single(lp, y, blank=0):
    """lp [T, U+1, V] (log-probs), y [U] -> (nll, grad [T, U+1, V] of nll w.r.t. lp)."""
    lp = np.asarray(lp, np.float64)
    T, U1, V = lp.shape
    U = U1 - 1
    y = np.asarray(y, np.int64)[:U]
    lb = lp[:, :, blank]
    ly = np.full((T, U1), -np.inf)
    if U:
        ly[:, :U] = lp[:, np.arange(U), y]
    a = np.full((T, U1), -np.inf)
    a[0, 0] = 0.0
    for t in range(T):
        for u in range(U1):
            if t == 0 and u == 0:
                continue
            c = []
            if t > 0:
                c.append(a[t - 1, u] + lb[t - 1, u])
            if u > 0:
                c.append(a[t, u - 1] + ly[t, u - 1])
            a[t, u] = np.logaddexp.reduce(c)
    b = np.full((T, U1), -np.inf)
    b[T - 1, U] = lb[T - 1, U]
    for t in range(T - 1, -1, -1):
        for u in range(U, -1, -1):
            if t == T - 1 and u == U:
                continue
            c = []
            if t < T - 1:
                c.append(b[t + 1, u] + lb[t, u])
            if u < U:
                c.append(b[t, u + 1] + ly[t, u])
            b[t, u] = np.logaddexp.reduce(c)
    logp = a[T - 1, U] + lb[T - 1, U]
    g = np.zeros_like(lp)
    gb = np.zeros((T, U1))
    gb[:T - 1] = -np.exp(a[:T - 1] + lb[:T - 1] + b[1:] - logp)
    gb[T - 1, U] = -np.exp(a[T - 1, U] + lb[T - 1, U] - logp)
    g[:, :, blank] += gb
    if U:
        gy = -np.exp(a[:, :U] + ly[:, :U] + b[:, 1:] - logp)
        for u in range(U):
            g[:, u, y[u]] += gy[:, u]
    return -logp, g


def brute_force_nll(lp, y, blank=0):
    """-log sum over all alignments: interleavings of T-1 blanks (one per frame advance, the last
    frame's final blank fixed) with the U labels."""
    lp = np.asarray(lp, np.float64)
    T, U1, _ = lp.shape
    U = U1 - 1
    tot = []
    for pos in itertools.combinations(range(T - 1 + U), U):   # positions of the labels
        t = u = 0
        s = 0.0
        for k in range(T - 1 + U):
            if k in pos:
                s += lp[t, u, y[u]]
                u += 1
            else:
                s += lp[t, u, blank]
                t += 1
        s += lp[T - 1, U, blank]
        tot.append(s)
    return -np.logaddexp.reduce(tot)


def rnnt_loss(log_probs, labels, frames_lengths, labels_lengths, blank=0, reduction="mean",
              average_frames=False):
    """Batched dense form (B, T, U+1, V) with warp_rnnt's reductions; returns (loss, costs,
    grad w.r.t. log_probs of the reduced loss)."""
    lp = np.asarray(log_probs, np.float64)
    B = lp.shape[0]
    costs = np.zeros(B)
    grad = np.zeros_like(lp)
    for b in range(B):
        T, U = int(frames_lengths[b]), int(labels_lengths[b])
        c, g = rnnt_single(lp[b, :T, :U + 1], labels[b, :U], blank)
        costs[b] = c
        grad[b, :T, :U + 1] = g
    scale = np.ones(B)
    if average_frames:
        scale = scale / np.asarray(frames_lengths, np.float64)
    if reduction == "mean":
        scale = scale / B
    elif reduction == "none":
        return costs * (1 / np.asarray(frames_lengths, np.float64) if average_frames else 1), costs, None
    return float((costs * scale).sum()), costs, grad * scale[:, None, None, None]
