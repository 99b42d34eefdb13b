#!/usr/bin/env python3
"""Golden fixtures for the mLSTM cell -> tests/golden/mlstm.npz.

The reference's xLSTM encoder comes from an external fork (speechcatcher-asr/xlstm +
mlstm_kernels) that is neither vendored nor installable offline: parity w.r.t. the fork is
UNPINNED.  The mLSTM math is pinned instead by the in-container HF transformers
5.15.0 native kernels (transformers/models/xlstm/modeling_xlstm.py:74-386, chunkwise form with
native autograd), which restate the same published algorithm.  Run here (CPU, fp64):

    python tests/golden/gen_mlstm.py

Stored per case: q, k, v [B,NH,T,D*], igate, fgate [B,NH,T] (pre-activations), optional
initial state (c0 [B,NH,DQ,DV], n0 [B,NH,DQ], m0 [B,NH,1]); outputs h [B,NH,T,DV] and final
state (cT, nT, mT); gradients of sum(h * R) w.r.t. every input (R stored).
"""
import os

import numpy as np
import torch
from transformers.models.xlstm import modeling_xlstm as M

HERE = os.path.dirname(os.path.abspath(__file__))


def case(B, NH, T, DQ, DV, seed, init=False):
    g = torch.Generator().manual_seed(seed)
    f64 = torch.float64
    q = torch.randn(B, NH, T, DQ, generator=g, dtype=f64)
    k = torch.randn(B, NH, T, DQ, generator=g, dtype=f64)
    v = torch.randn(B, NH, T, DV, generator=g, dtype=f64)
    ig = torch.randn(B, NH, T, generator=g, dtype=f64) * 3.0
    fg = torch.randn(B, NH, T, generator=g, dtype=f64) * 2.0 + 3.0
    ins = dict(q=q, k=k, v=v, igate=ig, fgate=fg)
    st = {}
    if init:
        st = dict(c0=torch.randn(B, NH, DQ, DV, generator=g, dtype=f64) * 0.5,
                  n0=torch.randn(B, NH, DQ, generator=g, dtype=f64) * 0.5,
                  m0=torch.randn(B, NH, 1, generator=g, dtype=f64))
    leaves = {n: t.clone().requires_grad_(True) for n, t in {**ins, **st}.items() if n != "m0"}
    h, (cT, nT, mT) = M.mlstm_chunkwise_native_autograd(
        leaves["q"], leaves["k"], leaves["v"], leaves["igate"], leaves["fgate"],
        c_initial=leaves.get("c0"), n_initial=leaves.get("n0"), m_initial=st.get("m0"),
        return_last_states=True, chunk_size=64)
    R = torch.randn(h.shape, generator=g, dtype=f64)
    (h * R).sum().backward()
    out = {n: t.numpy() for n, t in {**ins, **st}.items()}
    out.update(h=h.detach().numpy(), cT=cT.detach().numpy(), nT=nT.detach().numpy(),
               mT=mT.detach().numpy(), R=R.numpy())
    for n, t in leaves.items():
        out["d" + n] = t.grad.numpy()
    # inputs are exactly representable in fp32 only after rounding: store fp32 inputs and the
    # fp64 results computed from those rounded inputs would differ by ~1e-7; keep it simple and
    # store everything in fp32 (the GPU tolerances are >= 1e-4)
    return {k: v.astype(np.float32) for k, v in out.items()}


def block_case(seed=5):
    """One HF xLSTMBlock (hidden 128, 2 heads -> DQ 32, DV 64) in fp64: the layer/block
    structure statecatcher_amd/xlstm.py mirrors."""
    from transformers import xLSTMConfig
    cfg = xLSTMConfig(hidden_size=128, embedding_dim=128, num_heads=2, num_blocks=1, vocab_size=10,
                      mode="train", chunkwise_kernel="chunkwise--native_autograd",
                      autocast_kernel_dtype="float32", return_last_states=True)
    torch.manual_seed(seed)
    blk = M.xLSTMBlock(cfg).double()
    with torch.no_grad():
        for name, p in blk.named_parameters():
            if p.dim() > 1:
                p.normal_(0.0, 0.08)
            elif "norm" in name:
                p.normal_(1.0, 0.1)
            else:
                p.normal_(0.0, 1.0)
    x = torch.randn(2, 128, 128, dtype=torch.float64, requires_grad=True)
    y, (c, n, m) = blk(x)
    R = torch.randn(y.shape, dtype=torch.float64)
    (y * R).sum().backward()
    out = {"param/" + k: v.detach().numpy() for k, v in blk.state_dict().items()}
    out.update(x=x.detach().numpy(), y=y.detach().numpy(), cT=c.detach().numpy(),
               nT=n.detach().numpy(), mT=m.detach().numpy(), R=R.numpy(), dx=x.grad.numpy(),
               dq_weight=blk.mlstm_layer.q.weight.grad.numpy(),
               dfgate_bias=blk.mlstm_layer.fgate_preact.bias.grad.numpy())
    return {k: v.astype(np.float32) for k, v in out.items()}


def main():
    cases = {"small": case(1, 2, 128, 32, 64, 1), "state": case(2, 1, 64, 32, 64, 2, init=True),
             "c4": case(1, 1, 128, 96, 192, 3, init=True)}
    cases["block"] = block_case()
    flat = {f"{c}/{k}": v for c, d in cases.items() for k, v in d.items()}
    np.savez_compressed(os.path.join(HERE, "mlstm.npz"), **flat)
    print({k: v.shape for k, v in flat.items() if k.startswith("c4/")})


if __name__ == "__main__":
    main()
