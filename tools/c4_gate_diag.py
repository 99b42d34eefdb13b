#!/usr/bin/env python3
"""Diagnostic: the mLSTM gate-bias gradients of the C4 step, per cell path.

Runs tests/test_gpu_c4.py's C4 step (B = 2, T = 1500 -> 1536) three ways on the same weights:
bf16 cell through ops.MLSTMCoreFn, bf16 cell through the split path (mlstm_chunkwise), fp16
cell (split path).  Prints the igate / fgate bias gradients of every block and, for the last
block, checks the split path's cell against tests/torch_ref.mlstm64 in fp64 on the cell's own
(captured) rounded inputs and incoming dh.
usage: python tools/c4_gate_diag.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_c4 as c4   # noqa: E402
from statecatcher_amd import ops, xlstm   # noqa: E402

c4.DEV = torch.device("cuda:0")
CAP = {}
_orig_cell = xlstm.mlstm_chunkwise


def capturing_cell(q, k, v, ig, fg, c0, n0, m0, **kw):
    n = CAP.setdefault("_n", [0])
    n[0] += 1
    leaves = [t.detach().clone().requires_grad_(True) for t in (q, k, v, ig, fg)]
    h, _ = _orig_cell(*leaves, c0, n0, m0, **kw)    # a private graph on the captured inputs
    rec = {"in": leaves, "c0": c0, "n0": n0, "m0": m0, "h": h}
    CAP[n[0]] = rec
    h2, st2 = _orig_cell(q, k, v, ig, fg, c0, n0, m0, **kw)
    h2.register_hook(lambda g, rec=rec: rec.__setitem__("dh", g.detach().clone()))
    return h2, st2


def step(kdt, split, capture=False):
    init = STATE
    orig = ops.mlstm_core_supported
    if split:
        ops.mlstm_core_supported = lambda *a: False
    if capture:
        xlstm.mlstm_chunkwise = capturing_cell
    try:
        loss, grads, _, _ = c4.one_step(kdt, init)
    finally:
        ops.mlstm_core_supported = orig
        xlstm.mlstm_chunkwise = _orig_cell
    return loss, grads


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float(a @ b / max(float(a.norm() * b.norm()), 1e-300))


STATE = {k: v.detach().clone() for k, v in c4.c4_model("bfloat16").state_dict().items()}
runs = {"bf16-core": step("bfloat16", False), "bf16-split": step("bfloat16", True),
        "fp16-split": step("float16", True)}
for name, (loss, _) in runs.items():
    print(f"{name}: loss {loss:.5f}")
for blk in range(12):
    for g in ("igate", "fgate"):
        key = f"encoder.blocks.{blk}.mlstm_layer.{g}_preact.bias"
        vals = {n: r[1][key] for n, r in runs.items()}
        print(f"block {blk:2d} {g}: " + " | ".join(
            f"{n} {[round(float(x), 4) for x in v]}" for n, v in vals.items())
            + f" | cos core/split {cos(vals['bf16-core'], vals['bf16-split']):.3f}"
            f" split/fp16 {cos(vals['bf16-split'], vals['fp16-split']):.3f}")

# cell-level truth for the last block: capture the split path's inputs and dh
from tests.torch_ref import mlstm64   # noqa: E402
for kdt in ("bfloat16", "float16"):
    CAP.clear()
    step(kdt, True, capture=True)
    rec = CAP[max(k for k in CAP if k != "_n")]
    q, k, v, ig, fg = rec["in"]
    gq, gk, gv, gi, gf = torch.autograd.grad(rec["h"], rec["in"], rec["dh"])
    ref = [t.detach().double().requires_grad_(True) for t in (q, k, v, ig, fg)]
    B, NH, _, DQ = q.shape
    z = dict(device=q.device, dtype=torch.float64)
    extra = [torch.zeros(B, NH, DQ, v.shape[-1], **z), torch.zeros(B, NH, DQ, **z),
             torch.zeros(B, NH, 1, **z)]
    assert all(t is None for t in (rec["c0"], rec["n0"], rec["m0"]))
    rh, _ = mlstm64(*ref, *extra)
    (rh * rec["dh"].double()).sum().backward()
    for name, got, r in zip("q k v ig fg".split(), (gq, gk, gv, gi, gf), ref):
        rel = float((got.double() - r.grad).norm() / max(float(r.grad.norm()), 1e-300))
        print(f"last cell ({kdt}) d{name}: rel {rel:.3e}, cos {cos(got, r.grad):.4f}"
              + (f", bias-sum ours {[round(float(x), 4) for x in got.sum((0, 2))]} fp64 "
                 f"{[round(float(x), 4) for x in r.grad.sum((0, 2))]}" if name in ("ig", "fg") else ""))
