"""Native LucyRNN (reference lucyrnn.py) restated in numpy — TEST INFRASTRUCTURE ONLY.

Follows /root/reference/lucyrnn.py step by step, time loops included (small shapes only):
  * ``cell``            LucyRNNCell.forward, lucyrnn.py:44-70 (fused :47-54 / unfused :55-62,
                        mask blend :66-68)
  * ``lucyrnn_forward`` LucyRNN.forward, lucyrnn.py:89-191: frame stacking :92-99, train mode
                        :109-170 (decay scan with s_{-1} = 0, then the per-step cell fed the SCAN
                        state as s_prev, so decay is applied twice and s is never carried —
                        SURVEY F9), infer mode :172-184 (true recurrence), output projection.
Pinned by tests/golden/native.npz (reference lucyrnn.LucyRNN outputs).
"""
import numpy as np


def _sig(x):
    return 1.0 / (1.0 + np.exp(-x))


def _ln(x, p, name, on):
    if not on:
        return x
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + 1e-5) * p[name + ".weight"] + p[name + ".bias"]


def _lin(x, p, name):
    return x @ p[name + ".weight"].T + p[name + ".bias"]


def cell(p, pre, x, h_prev, s_prev, fused, ln, mask=None):
    """lucyrnn.py:44-70 for one step; p holds the layer's parameters, prefix `pre`."""
    u = _ln(_lin(x, p, pre + "input_proj"), p, pre + "layernorm_in", ln)
    if fused:
        r, z, k, v, h_pre, dl = np.split(_lin(u, p, pre + "W_fused"), 6, axis=-1)
        z = _sig(_ln(z, p, pre + "layernorm_z", ln))
        decay = _sig(dl)
        s = decay * s_prev + k * v
        c = np.tanh(_ln(h_pre + s, p, pre + "layernorm_h", ln))
    else:
        z = _sig(_ln(_lin(u, p, pre + "W_z"), p, pre + "layernorm_z", ln))
        k = _lin(u, p, pre + "W_k")
        v = _lin(u, p, pre + "W_v")
        decay = _sig(_lin(u, p, pre + "W_decay"))
        s = decay * s_prev + k * v
        c = np.tanh(_ln(_lin(u + s, p, pre + "W_h"), p, pre + "layernorm_h", ln))
    h = (1 - z) * c + z * h_prev
    if mask is not None:
        h = mask * h + (1 - mask) * h_prev
        s = mask * s + (1 - mask) * s_prev
    return h, s


def lucyrnn_forward(p, x, L, D, train, fused, ln, decay_mode="learned", stack=1,
                    lambda_decay=0.001, h0=None, s0=None):
    """lucyrnn.py:89-191 -> (logits, h list, s list)."""
    x = np.asarray(x, np.float64)
    B, T, F = x.shape
    if stack > 1:
        Tt = T - T % stack
        x = x[:, :Tt].reshape(B, Tt // stack, F * stack)
        T = x.shape[1]
    h = [np.zeros((B, D)) if h0 is None else np.array(h0[l], np.float64) for l in range(L)]
    s = [np.zeros((B, D)) if s0 is None else np.array(s0[l], np.float64) for l in range(L)]
    if train:
        inp = x
        for l in range(L):
            pre = f"layers.{l}."
            u = _ln(_lin(inp, p, pre + "input_proj"), p, pre + "layernorm_in", ln)
            if fused:
                _, _, k, v, _, dl = np.split(_lin(u, p, pre + "W_fused"), 6, axis=-1)
            else:
                k, v = _lin(u, p, pre + "W_k"), _lin(u, p, pre + "W_v")
                dl = _lin(u, p, pre + "W_decay")
            kv = k * v
            if decay_mode == "learned":
                decay = _sig(dl)
                s_all = np.zeros_like(kv)
                st = np.zeros((B, D))
                for t in range(T):
                    st = decay[:, t] * st + kv[:, t]
                    s_all[:, t] = st
            else:   # prefix_sum, lucyrnn.py:126-142
                tt = np.arange(T, dtype=np.float64)[None, :, None]
                dec = np.exp(np.broadcast_to(-lambda_decay * tt, (B, T, D)))
                lw = np.cumsum(np.log(dec + 1e-7), axis=1)
                s_all = np.cumsum(kv * np.exp(lw), axis=1) / (np.exp(lw) + 1e-7)
            out = np.zeros((B, T, D))
            for t in range(T):
                h[l], _ = cell(p, pre, inp[:, t], h[l], s_all[:, t], fused, ln)
                out[:, t] = h[l]
            inp = out
        outputs = inp
    else:
        outputs = np.zeros((B, T, D))
        for t in range(T):
            it = x[:, t]
            for l in range(L):
                h[l], s[l] = cell(p, f"layers.{l}.", it, h[l], s[l], fused, ln)
                it = h[l]
            outputs[:, t] = h[-1]
    logits = _lin(outputs, p, "output_proj")
    return logits, h, s
