"""Oracle (TEST INFRASTRUCTURE ONLY): numpy fp64 CTC alpha-beta.

The reference's CTC is ``nn.CTCLoss(blank=0, zero_infinity=True)`` (train.py:142) applied
to ``enc_out.log_softmax(-1).transpose(0, 1)`` (model.py:68-71), i.e. ATen's ``ctc_loss``
(a third-party dependency: torch, unpinned in requirements.txt:5).  This file restates the
published CTC forward-backward (Graves et al. 2006, eqs. 6-16) the way ATen's CPU kernel
computes it (log-space alpha/beta over the 2U+1 blank-extended states; gradient
``exp(lp) - exp(lcab + nll - lp)`` per label).  Pinned against ``torch.ctc_loss`` fp64 by
tests/golden/gen_golden.py.
"""
import numpy as np

NEG_INF = -np.inf


def _lse(*xs):
    m = np.max(np.stack(xs), axis=0)
    with np.errstate(invalid="ignore", divide="ignore"):
        safe = np.where(np.isfinite(m), m, 0.0)
        r = np.log(np.sum(np.exp(np.stack(xs) - safe), axis=0)) + safe
    return np.where(np.isneginf(m), NEG_INF, r)


def log_softmax(x):
    x = np.asarray(x, dtype=np.float64)
    m = x.max(axis=-1, keepdims=True)
    return x - (np.log(np.exp(x - m).sum(axis=-1, keepdims=True)) + m)


def ctc_single(lp, tgt, blank=0):
    """lp (T_b, V) log-probs, tgt (U,) ints -> nll, grad (T_b, V) wrt lp in ATen's convention.

    ATen's gradient for log-prob inputs is exp(lp) - exp(lcab + nll - lp), which equals the
    gradient w.r.t. the logits when lp = log_softmax(logits).
    """
    lp = np.asarray(lp, dtype=np.float64)
    T, V = lp.shape
    U = len(tgt)
    S = 2 * U + 1
    ext = np.full(S, blank, dtype=np.int64)
    ext[1::2] = tgt
    if T == 0:
        nll = 0.0 if U == 0 else np.inf
        return nll, np.zeros((0, V))
    # skip-transition allowed into state s from s-2 (non-blank and different label)
    skip = np.zeros(S, dtype=bool)
    skip[2:] = (ext[2:] != blank) & (ext[2:] != ext[:-2])
    alpha = np.full((T, S), NEG_INF)
    alpha[0, 0] = lp[0, ext[0]]
    if S > 1:
        alpha[0, 1] = lp[0, ext[1]]
    for t in range(1, T):
        a = alpha[t - 1]
        a1 = np.concatenate([[NEG_INF], a])[:S]
        a2 = np.concatenate([[NEG_INF, NEG_INF], a])[:S]
        a2 = np.where(skip, a2, NEG_INF)
        alpha[t] = _lse(a, a1, a2) + lp[t, ext]
    if S > 1:
        ll = _lse(alpha[T - 1, S - 1], alpha[T - 1, S - 2])
    else:
        ll = alpha[T - 1, 0]
    nll = -float(ll)
    beta = np.full((T, S), NEG_INF)
    beta[T - 1, S - 1] = lp[T - 1, ext[S - 1]]
    if S > 1:
        beta[T - 1, S - 2] = lp[T - 1, ext[S - 2]]
    skip_b = np.zeros(S, dtype=bool)            # transition s -> s+2 allowed
    skip_b[:-2] = skip[2:]
    for t in range(T - 2, -1, -1):
        b = beta[t + 1]
        b1 = np.concatenate([b, [NEG_INF]])[1:]
        b2 = np.concatenate([b, [NEG_INF, NEG_INF]])[2:]
        b2 = np.where(skip_b, b2, NEG_INF)
        beta[t] = _lse(b, b1, b2) + lp[t, ext]
    ab = alpha + beta
    lcab = np.full((T, V), NEG_INF)
    for s in range(S):
        lcab[:, ext[s]] = _lse(lcab[:, ext[s]], ab[:, s])
    with np.errstate(over="ignore", invalid="ignore"):
        grad = np.exp(lp) - np.exp(lcab + nll - lp)
    return nll, grad


def ctc_loss_grad(x, targets, in_lens, tgt_lens, blank=0, logits=True):
    """Batched CTC.

    x: (B, T, V) logits (``logits=True``; log_softmax applied here, as model.py:70 does) or
       log-probs (``logits=False``).
    targets: (B, Umax) padded, or a list of sequences.  Returns (nll (B,), grad (B,T,V)) where
    grad is the per-sample gradient of nll_b w.r.t. x (rows t >= in_len are zero).
    """
    x = np.asarray(x, dtype=np.float64)
    B, T, V = x.shape
    lp_all = log_softmax(x) if logits else x
    nll = np.zeros(B)
    grad = np.zeros((B, T, V))
    for b in range(B):
        Tb = int(in_lens[b])
        Ub = int(tgt_lens[b])
        tgt = np.asarray(targets[b][:Ub], dtype=np.int64)
        n, g = ctc_single(lp_all[b, :Tb], tgt, blank)
        nll[b] = n
        if Tb:
            grad[b, :Tb] = g
    return nll, grad


def ctc_mean_zero_inf(nll, tgt_lens):
    """Reduction of nn.CTCLoss(reduction='mean', zero_infinity=True): mean_b(nll_b / max(U_b,1))."""
    nll = np.where(np.isinf(nll), 0.0, nll)
    return float(np.mean(nll / np.maximum(np.asarray(tgt_lens, dtype=np.float64), 1.0)))


def ctc_mean_grad_scale(nll, tgt_lens):
    """d loss / d nll_b for the 'mean' + zero_infinity reduction."""
    B = len(nll)
    sc = 1.0 / (B * np.maximum(np.asarray(tgt_lens, dtype=np.float64), 1.0))
    return np.where(np.isinf(nll), 0.0, sc)
