"""mLSTM cell (xLSTM matrix memory) restated in numpy — TEST INFRASTRUCTURE ONLY.

The reference's xLSTM encoder (model.py:214-229, :301-307) comes from an external fork that is
not available here (parity w.r.t. the fork unpinned).  This restates the published
mLSTM recurrence as the in-container HF transformers 5.15.0 native step kernel does
(transformers/models/xlstm/modeling_xlstm.py:388-449, ``mlstm_recurrent_step_native``), per
head, with the stabiliser m:
    m_t = max(logsig(f_t) + m_{t-1}, i_t)
    C_t = e^{logsig(f_t) + m_{t-1} - m_t} C_{t-1} + e^{i_t - m_t} k_t v_t^T
    n_t = e^{logsig(f_t) + m_{t-1} - m_t} n_{t-1} + e^{i_t - m_t} k_t
    h_t = (q_t s C_t) / (max(|q_t s . n_t|, e^{-m_t}) + eps),  s = DQ^-1/2
Pinned against tests/golden/mlstm.npz (HF chunkwise native autograd, fp64).
"""
import numpy as np


def _logsig(x):
    return -np.logaddexp(0.0, -x)


def mlstm_recurrent(q, k, v, igate, fgate, c0=None, n0=None, m0=None, eps=1e-6):
    """q, k [B,NH,T,DQ], v [B,NH,T,DV], gates [B,NH,T] -> h [B,NH,T,DV], (C, n, m) final."""
    q, k, v = (np.asarray(a, np.float64) for a in (q, k, v))
    ig, fg = np.asarray(igate, np.float64), np.asarray(fgate, np.float64)
    B, NH, T, DQ = q.shape
    DV = v.shape[-1]
    C = np.zeros((B, NH, DQ, DV)) if c0 is None else np.array(c0, np.float64)
    n = np.zeros((B, NH, DQ)) if n0 is None else np.array(n0, np.float64)
    m = np.zeros((B, NH)) if m0 is None else np.array(m0, np.float64).reshape(B, NH)
    s = DQ ** -0.5
    h = np.zeros((B, NH, T, DV))
    for t in range(T):
        lf = _logsig(fg[..., t])
        mn = np.maximum(lf + m, ig[..., t])
        fa = np.exp(lf + m - mn)[..., None]
        ia = np.exp(ig[..., t] - mn)[..., None]
        C = fa[..., None] * C + ia[..., None] * (k[..., t, :, None] * v[..., t, None, :])
        n = fa * n + ia * k[..., t, :]
        qs = q[..., t, :] * s
        num = np.einsum("bhi,bhij->bhj", qs, C)
        den = np.maximum(np.abs((qs * n).sum(-1)), np.exp(-mn)) + eps
        h[..., t, :] = num / den[..., None]
        m = mn
    return h, (C, n, m[..., None])
