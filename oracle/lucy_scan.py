"""Oracle (TEST INFRASTRUCTURE ONLY): numpy restatement of the LucyRNN gated scan.

Forward follows /root/reference/lucyrnn_triton.py:179-244 (``rnn_forward_unfused_rmsnorm``)
operation by operation; ``decay_scan`` follows lucyrnn_triton.py:158-177
(``fused_decay_scan``).  The backward has no counterpart in the reference (SURVEY F2:
its outputs carry no grad_fn); ``lucy_scan_bwd`` is the analytic adjoint of the
forward and is pinned by torch.autograd of an fp64 restatement (tests/golden).

All functions are vectorised over (B, D) and loop over T, computing in ``dtype``
(float64 by default).
"""
import numpy as np

EPS = 1e-6  # lucyrnn_triton.py:214-218, :235


def _sig(x):
    with np.errstate(over="ignore"):
        return 1.0 / (1.0 + np.exp(-x))


def _planes(g):
    # gate order r, z, k, v, h_pre, decay, alpha — lucyrnn_triton.py:205-211
    return [g[:, i, :] for i in range(7)]


def _step_terms(g, dtype):
    """Per-step elementwise terms of lucyrnn_triton.py:213-235 for one time step."""
    r, z, k, v, hp, dc, al = [p.astype(dtype) for p in _planes(g)]
    eps = dtype(EPS)
    two = dtype(2)
    rc = np.sqrt((r * r + z * z) / two + eps)      # :214
    rkv = np.sqrt((k * k + v * v) / two + eps)     # :215
    rd = np.sqrt(dc * dc + eps)                    # :216
    ra = np.sqrt(al * al + eps)                    # :217
    rh = np.sqrt(hp * hp + eps)                    # :218
    zg = _sig(z / rc)                              # :221, :230
    dec = _sig(dc / rd)                            # :222, :231
    kn = k / rkv                                   # :223
    vn = v / rkv                                   # :224
    hn = hp / rh                                   # :225
    alp = _sig(al / ra)                            # :226, :232
    kv = (kn * vn) / (rkv * rkv + eps)             # :235
    return zg, dec, alp, kv, hn


def lucy_scan_fwd(gates, h0, s0, dtype=np.float64):
    """gates (B,T,7,D), h0/s0 (B,D) -> out (B,T,D), s_last (B,D)."""
    gates = np.asarray(gates)
    B, T, G, D = gates.shape
    assert G == 7
    h = np.asarray(h0, dtype=dtype).copy()
    s = np.asarray(s0, dtype=dtype).copy()
    out = np.empty((B, T, D), dtype=dtype)
    two = dtype(2)
    one = dtype(1)
    for t in range(T):
        zg, dec, alp, kv, hn = _step_terms(gates[:, t], dtype)
        s = dec * s + alp * kv                     # :238
        c = _sig(two * (hn + s)) * two - one       # :239
        h = (one - zg) * c + zg * h                # :240
        out[:, t] = h                              # :242
    return out, s                                  # :244


def lucy_scan_bwd(gates, h0, s0, dout, ds_last, dtype=np.float64):
    """Adjoint of ``lucy_scan_fwd``.

    dout (B,T,D) = dL/d out, ds_last (B,D) = dL/d s_last.
    Returns dgates (B,T,7,D), dh0 (B,D), ds0 (B,D).

    Recurrences (reverse time):
      Gh_t = dout_t + zg_{t+1} Gh_{t+1}
      Gs_t = Gh_t (1-zg_t)(1-c_t^2) + dec_{t+1} Gs_{t+1},  Gs_{T-1} += ds_last
    """
    gates = np.asarray(gates, dtype=dtype)
    B, T, _, D = gates.shape
    eps = dtype(EPS)
    two = dtype(2)
    one = dtype(1)
    # forward recompute, keeping every state
    hs = np.empty((T + 1, B, D), dtype=dtype)
    ss = np.empty((T + 1, B, D), dtype=dtype)
    cs = np.empty((T, B, D), dtype=dtype)
    hs[0] = h0
    ss[0] = s0
    for t in range(T):
        zg, dec, alp, kv, hn = _step_terms(gates[:, t], dtype)
        ss[t + 1] = dec * ss[t] + alp * kv
        cs[t] = _sig(two * (hn + ss[t + 1])) * two - one
        hs[t + 1] = (one - zg) * cs[t] + zg * hs[t]
    dgates = np.empty_like(gates)
    carry_h = np.zeros((B, D), dtype=dtype)                 # zg_{t+1} Gh_{t+1}
    carry_s = np.asarray(ds_last, dtype=dtype).copy()       # dec_{t+1} Gs_{t+1}
    dout = np.asarray(dout, dtype=dtype)
    for t in range(T - 1, -1, -1):
        r, z, k, v, hp, dc, al = _planes(gates[:, t])
        zg, dec, alp, kv, hn = _step_terms(gates[:, t], dtype)
        c = cs[t]
        gh = dout[:, t] + carry_h
        dpre = gh * (one - zg) * (one - c * c)
        gs = dpre + carry_s
        d_zg = gh * (hs[t] - c)
        d_dec = gs * ss[t]
        d_alp = gs * kv
        d_kv = gs * alp
        # sigmoid inputs
        d_zn = d_zg * zg * (one - zg)
        d_dn = d_dec * dec * (one - dec)
        d_an = d_alp * alp * (one - alp)
        # per-element rms normalisers x / sqrt(x^2 + eps): derivative eps / rho^3
        rd2 = dc * dc + eps
        ra2 = al * al + eps
        rh2 = hp * hp + eps
        d_dc = d_dn * eps / (rd2 * np.sqrt(rd2))
        d_al = d_an * eps / (ra2 * np.sqrt(ra2))
        d_hp = dpre * eps / (rh2 * np.sqrt(rh2))
        # zn = z / rho_c, rho_c^2 = (r^2+z^2)/2 + eps
        rc2 = (r * r + z * z) / two + eps
        rc3 = rc2 * np.sqrt(rc2)
        d_z = d_zn * (r * r / two + eps) / rc3
        d_r = -d_zn * z * r / (two * rc3)
        # kv = k v / (q (q+eps)),  q = (k^2+v^2)/2 + eps
        q = (k * k + v * v) / two + eps
        f = one / (q * (q + eps))
        fp = -(two * q + eps) * f * f
        d_k = d_kv * (v * f + k * k * v * fp)
        d_v = d_kv * (k * f + k * v * v * fp)
        dgates[:, t, 0] = d_r
        dgates[:, t, 1] = d_z
        dgates[:, t, 2] = d_k
        dgates[:, t, 3] = d_v
        dgates[:, t, 4] = d_hp
        dgates[:, t, 5] = d_dc
        dgates[:, t, 6] = d_al
        carry_h = zg * gh
        carry_s = dec * gs
    return dgates, carry_h, carry_s


def decay_scan(kv, decay, dtype=np.float32):
    """lucyrnn_triton.py:158-177: s_t = decay_t * s_{t-1} + kv_t, s_{-1} = 0 (fp32 acc :171)."""
    kv = np.asarray(kv)
    decay = np.asarray(decay)
    B, T, D = kv.shape
    out = np.empty((B, T, D), dtype=dtype)
    s = np.zeros((B, D), dtype=dtype)
    for t in range(T):
        s = decay[:, t].astype(dtype) * s + kv[:, t].astype(dtype)
        out[:, t] = s
    return out


def decay_scan_bwd(decay, s_all, dout, dtype=np.float64):
    """Adjoint of ``decay_scan``: returns (dkv, ddecay)."""
    decay = np.asarray(decay, dtype=dtype)
    s_all = np.asarray(s_all, dtype=dtype)
    dout = np.asarray(dout, dtype=dtype)
    B, T, D = decay.shape
    dkv = np.empty((B, T, D), dtype=dtype)
    ddec = np.empty((B, T, D), dtype=dtype)
    carry = np.zeros((B, D), dtype=dtype)
    for t in range(T - 1, -1, -1):
        g = dout[:, t] + carry
        dkv[:, t] = g
        ddec[:, t] = g * (s_all[:, t - 1] if t > 0 else 0.0)
        carry = decay[:, t] * g
    return dkv, ddec
