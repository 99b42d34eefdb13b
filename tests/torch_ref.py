"""fp64 torch restatements used as autograd checkers by the GPU tests (test infrastructure).

scan64 restates lucyrnn_triton.py:204-242 exactly as tests/golden/gen_golden.py does (that
restatement is pinned against the reference Triton kernel by tests/test_oracle_golden.py);
lucyrnn64 composes it the way LucyRNNtriton.forward does (lucyrnn_triton.py:111-155).
"""
import torch


def scan64(gates, h0, s0):
    eps = 1e-6
    h, s = h0, s0
    outs = []
    for t in range(gates.shape[1]):
        r, z, k, v, hp, dc, al = [gates[:, t, i] for i in range(7)]
        rc = torch.sqrt((r * r + z * z) / 2 + eps)
        rkv = torch.sqrt((k * k + v * v) / 2 + eps)
        zg = torch.sigmoid(z / rc)
        dec = torch.sigmoid(dc / torch.sqrt(dc * dc + eps))
        alp = torch.sigmoid(al / torch.sqrt(al * al + eps))
        hn = hp / torch.sqrt(hp * hp + eps)
        kv = (k / rkv) * (v / rkv) / (rkv * rkv + eps)
        s = dec * s + alp * kv
        c = torch.sigmoid(2 * (hn + s)) * 2 - 1
        h = (1 - zg) * c + zg * h
        outs.append(h)
    return torch.stack(outs, 1), s


def lucyrnn64(params, x, L, D, states=None):
    """params: dict of fp64 leaf tensors named like LucyRNNtriton.state_dict()."""
    B, T, _ = x.shape
    h = [torch.zeros(B, D, dtype=x.dtype) for _ in range(L)] if states is None else list(states[0])
    s = [torch.zeros(B, D, dtype=x.dtype) for _ in range(L)] if states is None else list(states[1])
    for l in range(L):
        W = params[f"tracks.0.{l}.linear.weight"]
        bb = params[f"tracks.0.{l}.linear.bias"]
        gates = (x.reshape(B * T, -1) @ W.t() + bb).view(B, T, 7, D)
        x, s[l] = scan64(gates, h[l], s[l])
        h[l] = x[:, -1]
        if l < L - 1:
            x = torch.nn.functional.layer_norm(x, (D,), params[f"norms.0.{l}.weight"],
                                               params[f"norms.0.{l}.bias"], 1e-5)
    logits = x @ params["output_proj.weight"].t() + params["output_proj.bias"]
    return logits, (h, s)


def mlstm64(q, k, v, ig, fg, c0=None, n0=None, m0=None, eps=1e-6):
    """fp64 torch restatement of the mLSTM step recurrence (oracle/mlstm.py, itself pinned to
    transformers' chunkwise mLSTM by tests/test_oracle_golden.py), for autograd gradients."""
    B, NH, T, DQ = q.shape
    DV = v.shape[-1]
    C = torch.zeros(B, NH, DQ, DV, dtype=q.dtype) if c0 is None else c0
    n = torch.zeros(B, NH, DQ, dtype=q.dtype) if n0 is None else n0
    m = torch.zeros(B, NH, dtype=q.dtype) if m0 is None else m0.reshape(B, NH)
    s = DQ ** -0.5
    hs = []
    for t in range(T):
        lf = torch.nn.functional.logsigmoid(fg[..., t])
        mn = torch.maximum(lf + m, ig[..., t]).detach()   # the stabiliser is not differentiated
        fa = torch.exp(lf + m - mn)
        ia = torch.exp(ig[..., t] - mn)
        C = fa[..., None, None] * C + ia[..., None, None] * (k[..., t, :, None] * v[..., t, None, :])
        n = fa[..., None] * n + ia[..., None] * k[..., t, :]
        qs = q[..., t, :] * s
        num = torch.einsum("bhi,bhij->bhj", qs, C)
        den = torch.maximum((qs * n).sum(-1).abs(), torch.exp(-mn)) + eps
        hs.append(num / den[..., None])
        m = mn
    return torch.stack(hs, 2), (C, n, m[..., None])
