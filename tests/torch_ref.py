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
