"""Oracle (TEST INFRASTRUCTURE / CPU BASELINE ONLY): one LucyRNN + CTC training step in numpy.

The reference training step (train.py:529-571 -> model.py:37-110 -> lucyrnn_triton.py:111-155)
restated on the host: per layer GEMM (LinearSafe, :20-25) -> scan (oracle.lucy_scan, fp32) ->
LayerNorm (eps 1e-5, :96-97, :136-137); output projection; CTC 'mean' + zero_infinity
(oracle.ctc); the backward of all of it; clip_grad_norm_(50) and one Adam(lr 3e-4) update.
Used by bench.py as the `cpu_baseline` ("port") and by tests as a model-level checker.
"""
import numpy as np

from . import ctc as octc
from . import lucy_scan as oscan

LN_EPS = 1e-5


def init_params(L, Din, D, V, seed=0, out_std=0.02):
    rng = np.random.default_rng(seed)
    p = {}
    for l in range(L):
        din = Din if l == 0 else D
        a = np.sqrt(6.0 / (din + 7 * D))
        p[f"W{l}"] = rng.uniform(-a, a, (7 * D, din)).astype(np.float32)
        b = np.zeros((7, D), np.float32)
        b[1], b[5], b[6] = 1.0, 2.0, 0.5        # lucyrnn_triton.py:41-48
        p[f"b{l}"] = b.reshape(-1)
        if l < L - 1:
            p[f"g{l}"] = np.ones(D, np.float32)
            p[f"be{l}"] = np.zeros(D, np.float32)
    p["Wo"] = (rng.standard_normal((V, D)) * out_std).astype(np.float32)
    p["bo"] = np.zeros(V, np.float32)
    return p


def _ln_fwd(x, g, b):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    rstd = 1.0 / np.sqrt(var + LN_EPS)
    xh = (x - mu) * rstd
    return xh * g + b, (xh, rstd)


def _ln_bwd(dy, g, cache):
    xh, rstd = cache
    D = xh.shape[-1]
    dxh = dy * g
    dx = rstd / D * (D * dxh - dxh.sum(-1, keepdims=True) - xh * (dxh * xh).sum(-1, keepdims=True))
    return dx, (dy * xh).reshape(-1, D).sum(0), dy.reshape(-1, D).sum(0)


def forward(p, feats, L, D, state=None):
    """LucyRNNtriton.forward (lucyrnn_triton.py:111-155) with one track: per layer GEMM + bias
    (:20-25, :56) -> scan (fp32 state) -> h carry = out[:, -1] (:135) -> LayerNorm for l < L-1
    (:136-137); output_proj (:150).  Returns (logits, (h list, s list), x_last, caches)."""
    B, T, _ = feats.shape
    f32 = np.float32
    h = [np.zeros((B, D), f32)] * L if state is None else state[0]
    s = [np.zeros((B, D), f32)] * L if state is None else state[1]
    x = feats.astype(f32)
    caches = []
    new_h, new_s = [], []
    for l in range(L):
        gates = (x.reshape(-1, x.shape[-1]) @ p[f"W{l}"].T + p[f"b{l}"]).reshape(B, T, 7, D)
        out, s_last = oscan.lucy_scan_fwd(gates, h[l], s[l], dtype=f32)
        new_h.append(out[:, -1].copy())
        new_s.append(s_last)
        ln = None
        xin = x
        if l < L - 1:
            x, ln = _ln_fwd(out, p[f"g{l}"], p[f"be{l}"])
        else:
            x = out
        caches.append((xin, gates, ln))
    logits = x.reshape(-1, D) @ p["Wo"].T + p["bo"]
    return logits.reshape(B, T, -1), (new_h, new_s), x, (caches, h, s)


def train_step(p, feats, tokens, in_lens, tgt_lens, L, D, state=None, adam=None, lr=3e-4,
               max_norm=50.0):
    """One segment step: forward, CTC, backward, clip, Adam (updates p in place).
    Returns (loss, new_state, grads before clipping, adam state)."""
    B, T, _ = feats.shape
    f32 = np.float32
    logits, (new_h, new_s), x, (caches, h, s) = forward(p, feats, L, D, state)
    nll, grad = octc.ctc_loss_grad(logits, tokens, in_lens, tgt_lens, blank=0, logits=True)
    loss = octc.ctc_mean_zero_inf(nll, tgt_lens)
    scale = octc.ctc_mean_grad_scale(nll, tgt_lens)
    dlog = (np.where(np.isfinite(nll)[:, None, None], grad, 0.0) * scale[:, None, None]).astype(f32)
    gr = {"Wo": dlog.reshape(-1, dlog.shape[-1]).T @ x.reshape(-1, D), "bo": dlog.sum((0, 1))}
    dx = (dlog.reshape(-1, dlog.shape[-1]) @ p["Wo"]).reshape(B, T, D)
    for l in range(L - 1, -1, -1):
        xin, gates, ln = caches[l]
        if ln is not None:
            dx, gr[f"g{l}"], gr[f"be{l}"] = _ln_bwd(dx, p[f"g{l}"], ln)
        dg, _, _ = oscan.lucy_scan_bwd(gates, h[l], s[l], dx, np.zeros((B, D)), dtype=f32)
        dg2 = dg.reshape(-1, 7 * D).astype(f32)
        gr[f"W{l}"] = dg2.T @ xin.reshape(-1, xin.shape[-1])
        gr[f"b{l}"] = dg2.sum(0)
        dx = (dg2 @ p[f"W{l}"]).reshape(B, T, -1)
    # clip_grad_norm_(max_norm) (train.py:553) + Adam (train.py:133-136, 566)
    tot = np.sqrt(sum(float((g.astype(np.float64) ** 2).sum()) for g in gr.values()))
    coef = min(1.0, max_norm / (tot + 1e-6))
    if adam is None:
        adam = {"t": 0, "m": {k: np.zeros_like(v) for k, v in p.items()},
                "v": {k: np.zeros_like(v) for k, v in p.items()}}
    adam["t"] += 1
    b1, b2, eps = 0.9, 0.999, 1e-8
    for k, g in gr.items():
        g = (g * coef).astype(f32)
        adam["m"][k] = b1 * adam["m"][k] + (1 - b1) * g
        adam["v"][k] = b2 * adam["v"][k] + (1 - b2) * g * g
        mh = adam["m"][k] / (1 - b1 ** adam["t"])
        vh = adam["v"][k] / (1 - b2 ** adam["t"])
        p[k] -= (lr * mh / (np.sqrt(vh) + eps)).astype(f32)
    return loss, (new_h, new_s), gr, adam
