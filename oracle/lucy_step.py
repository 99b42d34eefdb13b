"""Oracle (TEST INFRASTRUCTURE / CPU BASELINE ONLY): one LucyRNN + CTC (C2) or RNN-T (C5)
training step in numpy.

The reference training step (train.py:529-571 -> model.py:37-110 -> lucyrnn_triton.py:111-155)
restated on the host: per layer GEMM (LinearSafe, :20-25) -> scan (oracle.lucy_scan, fp32) ->
LayerNorm (eps 1e-5, :96-97, :136-137); output projection; CTC 'mean' + zero_infinity
(oracle.ctc); the backward of all of it; clip_grad_norm_(50) and one Adam(lr 3e-4) update.
RNN-T (``rnnt_step``): RNNTPredictorJoiner (model.py:112-145) + log_softmax (model.py:93) +
the transducer lattice of warp_rnnt (train.py:38-42, gather=True; oracle.rnnt restates it and is
pinned by brute-force alignment sums) in fp64, the encoder as above.
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


def encoder_backward(p, dlog, x, caches, h, s, L, D):
    """Gradients of every encoder parameter from dL/dlogits (the backward of ``forward``):
    output_proj, then per layer (last first) LayerNorm -> scan (oracle.lucy_scan) -> gate GEMM."""
    B, T = dlog.shape[:2]
    f32 = np.float32
    dlog = dlog.astype(f32)
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
    return gr


def clip_and_adam(p, gr, adam=None, lr=3e-4, max_norm=50.0):
    """clip_grad_norm_(max_norm) (train.py:553) + Adam (train.py:133-136, 566), in place on p."""
    f32 = np.float32
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
    return adam


def train_step(p, feats, tokens, in_lens, tgt_lens, L, D, state=None, adam=None, lr=3e-4,
               max_norm=50.0):
    """One segment step: forward, CTC, backward, clip, Adam (updates p in place).
    Returns (loss, new_state, grads before clipping, adam state)."""
    f32 = np.float32
    logits, (new_h, new_s), x, (caches, h, s) = forward(p, feats, L, D, state)
    nll, grad = octc.ctc_loss_grad(logits, tokens, in_lens, tgt_lens, blank=0, logits=True)
    loss = octc.ctc_mean_zero_inf(nll, tgt_lens)
    scale = octc.ctc_mean_grad_scale(nll, tgt_lens)
    dlog = (np.where(np.isfinite(nll)[:, None, None], grad, 0.0) * scale[:, None, None]).astype(f32)
    gr = encoder_backward(p, dlog, x, caches, h, s, L, D)
    adam = clip_and_adam(p, gr, adam, lr, max_norm)
    return loss, (new_h, new_s), gr, adam


# ------------------------------------------------------------------------------ RNN-T (C5) ---
def _bf16(a):
    """Round to bf16 (nearest even) and back: the fused joiner's MFMA operand rounding."""
    a32 = np.ascontiguousarray(a, np.float32)
    u = a32.view(np.uint32).astype(np.uint64)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return u.astype(np.uint32).view(np.float32).astype(np.float64)


def rnnt_lattice(lb, ly):
    """Transducer alpha / beta over one sequence's (T, U+1) nodes, vectorised along the
    anti-diagonals (t + u = d): lb [T, U+1] blank log-probs, ly [T, U] next-label log-probs
    (oracle.rnnt.rnnt_single's recursion).  Returns (nll, d nll / d lb, d nll / d ly)."""
    T, U1 = lb.shape
    U = U1 - 1
    a = np.full((T, U1), -np.inf)
    b = np.full((T, U1), -np.inf)
    a[0, 0] = 0.0
    for d in range(1, T + U):
        u = np.arange(max(0, d - T + 1), min(U, d) + 1)
        t = d - u
        c1 = np.where(t > 0, a[np.maximum(t - 1, 0), u] + lb[np.maximum(t - 1, 0), u], -np.inf)
        c2 = np.where(u > 0, a[t, np.maximum(u - 1, 0)] + ly[t, np.maximum(u - 1, 0)], -np.inf) \
            if U else np.full(len(u), -np.inf)
        a[t, u] = np.logaddexp(c1, c2)
    b[T - 1, U] = lb[T - 1, U]
    for d in range(T + U - 2, -1, -1):
        u = np.arange(max(0, d - T + 1), min(U, d) + 1)
        t = d - u
        c1 = np.where(t < T - 1, b[np.minimum(t + 1, T - 1), u] + lb[t, u], -np.inf)
        c2 = np.where(u < U, b[t, np.minimum(u + 1, U)] + ly[t, np.minimum(u, U - 1)] if U else -np.inf,
                      -np.inf)
        b[t, u] = np.logaddexp(c1, c2)
    logp = a[T - 1, U] + lb[T - 1, U]
    gb = np.zeros((T, U1))
    gb[:T - 1] = -np.exp(a[:T - 1] + lb[:T - 1] + b[1:] - logp)
    gb[T - 1, U] = -np.exp(a[T - 1, U] + lb[T - 1, U] - logp)
    gy = -np.exp(a[:, :U] + ly + b[:, 1:] - logp) if U else np.zeros((T, 0))
    return -logp, gb, gy


def rnnt_joint_loss_grad(enc_p, pred_p, Wj, bj, labels, in_lens, tgt_lens, blank=0,
                         round_bf16=False, t_chunk=64):
    """RNNTPredictorJoiner's joint (model.py:129-145: z = tanh(enc_p + pred_p), logits = z Wj^T
    + bj) -> log_softmax -> transducer loss per sequence (warp_rnnt, gather=True), in fp64.
    Returns (nll [B], d enc_p, d pred_p, d Wj, d bj) of sum_b nll_b.  The (T, U+1, V) logits
    are formed t_chunk frames at a time (fp64 torch tensors on the CPU, for its threaded
    elementwise kernels; the lattice is rnnt_lattice).  round_bf16 rounds z and Wj to bf16 as the
    fused HIP joiner does (identity gradients)."""
    import torch
    f64 = torch.float64
    enc_p = torch.as_tensor(np.asarray(enc_p, np.float64))
    pred_p = torch.as_tensor(np.asarray(pred_p, np.float64))
    W = torch.as_tensor(_bf16(Wj) if round_bf16 else np.asarray(Wj, np.float64))
    bias = torch.as_tensor(np.asarray(bj, np.float64))
    rnd = (lambda z: z.to(torch.bfloat16).to(f64)) if round_bf16 else (lambda z: z)
    B = enc_p.shape[0]
    nll = np.zeros(B)
    de, dp = torch.zeros_like(enc_p), torch.zeros_like(pred_p)
    dW, db = torch.zeros_like(W), torch.zeros_like(bias)
    for bi in range(B):
        T, U = int(in_lens[bi]), int(tgt_lens[bi])
        if T == 0:
            nll[bi] = np.inf
            continue
        y = torch.as_tensor(np.asarray(labels[bi, :U], np.int64))
        lb = np.empty((T, U + 1))
        ly = np.empty((T, U))
        lses = []
        for t0 in range(0, T, t_chunk):
            t1 = min(T, t0 + t_chunk)
            z = torch.tanh(enc_p[bi, t0:t1, None, :] + pred_p[bi, None, :U + 1, :])
            lg = rnd(z) @ W.T + bias
            lse = torch.logsumexp(lg, -1)
            lses.append(lse)
            lb[t0:t1] = (lg[..., blank] - lse).numpy()
            if U:
                ly[t0:t1] = (lg[:, torch.arange(U), y] - lse[:, :U]).numpy()
        nll[bi], gb, gy = rnnt_lattice(lb, ly)
        gb, gy = torch.as_tensor(gb), torch.as_tensor(gy)
        for k, t0 in enumerate(range(0, T, t_chunk)):
            t1 = min(T, t0 + t_chunk)
            z = torch.tanh(enc_p[bi, t0:t1, None, :] + pred_p[bi, None, :U + 1, :])
            zq = rnd(z)
            lg = zq @ W.T + bias
            pr = torch.exp(lg - lses[k][..., None])
            g = torch.zeros_like(lg)                    # d nll / d log_probs (gathered arcs)
            g[..., blank] = gb[t0:t1]
            if U:
                g[:, torch.arange(U), y] += gy[t0:t1]
            dlg = g - pr * g.sum(-1, keepdim=True)      # through log_softmax
            dW += dlg.reshape(-1, dlg.shape[-1]).T @ zq.reshape(-1, zq.shape[-1])
            db += dlg.sum((0, 1))
            dpre = (dlg @ W) * (1.0 - z * z)
            de[bi, t0:t1] += dpre.sum(1)
            dp[bi, :U + 1] += dpre.sum(0)
    return nll, de.numpy(), dp.numpy(), dW.numpy(), db.numpy()


def rnnt_step(p, jp, feats, tokens, in_lens, tgt_lens, L, D, blank=0, round_bf16=False):
    """The C5 segment step up to the gradients: LucyRNNtriton forward (enc_out = logits, V-wide),
    RNNTPredictorJoiner (jp: emb [V,E], We [J,V], be [J], Wp [J,E], bp [J], Wj [V,J], bj [V];
    model.py:112-145), blank-prefixed predictor input (model.py:78-83), warp_rnnt 'mean' loss;
    then the backward of all of it.  Returns (loss, encoder grads, joiner grads)."""
    logits, _, x, (caches, h, s) = forward(p, feats, L, D)
    B, T, V = logits.shape
    prefix = np.concatenate([np.full((B, 1), blank, np.int64), np.asarray(tokens, np.int64)], 1)
    enc = logits.astype(np.float64)
    enc_p = enc @ jp["We"].T.astype(np.float64) + jp["be"]
    emb = jp["emb"].astype(np.float64)[prefix]
    pred_p = emb @ jp["Wp"].T.astype(np.float64) + jp["bp"]
    nll, de, dp, dWj, dbj = rnnt_joint_loss_grad(enc_p, pred_p, jp["Wj"], jp["bj"], tokens, in_lens,
                                                 tgt_lens, blank, round_bf16)
    loss = float(nll.mean())
    de /= B
    dp /= B
    jg = {"Wj": dWj / B, "bj": dbj / B,
          "We": de.reshape(-1, de.shape[-1]).T @ enc.reshape(-1, V), "be": de.sum((0, 1)),
          "Wp": dp.reshape(-1, dp.shape[-1]).T @ emb.reshape(-1, emb.shape[-1]), "bp": dp.sum((0, 1))}
    demb = dp @ jp["Wp"].astype(np.float64)
    g_emb = np.zeros(jp["emb"].shape)
    np.add.at(g_emb, prefix.reshape(-1), demb.reshape(-1, demb.shape[-1]))
    jg["emb"] = g_emb
    dlog = de @ jp["We"].astype(np.float64)
    gr = encoder_backward(p, dlog.astype(np.float32), x, caches, h, s, L, D)
    return loss, gr, jg
