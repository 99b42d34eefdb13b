"""Diagnostic (GPU): does sc_rnnt_joint_fwd / _bwd read outside one of its buffers?  Each buffer in
turn is placed at the start (then at the end) of a larger allocation whose rest holds garbage
(NaN for floats, huge values for integers); the results must not change."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from statecatcher_amd import _lib  # noqa: E402
from statecatcher_amd._lib import ptr, stream_of  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
B, T, U, V, J = int(sys.argv[1]) if len(sys.argv) > 1 else 2, 200, 12, 256, 64
enc = torch.randn(B, T, J, device=dev) * 0.5
pred = torch.randn(B, U + 1, J, device=dev) * 0.5
W = (torch.randn(V, J, device=dev) * 0.1).to(torch.bfloat16)
bias = torch.randn(V, device=dev) * 0.1
lens = torch.tensor([12, 7, 9, 12][:B], device=dev)
labels = torch.randint(1, V, (B, U), device=dev)
for b in range(B):
    labels[b, lens[b]:] = 0
flen = torch.full((B,), T, device=dev, dtype=torch.int64)
llen = lens.to(torch.int64)
lib = _lib.load()
wsb = lib.sc_rnnt_workspace_bytes(B, T, U)
PAD = 1 << 16   # elements of garbage around a buffer


def embed(t, where):
    """t's values inside a larger buffer of garbage; where = 'start' | 'end'."""
    n = t.numel()
    if t.dtype.is_floating_point:
        big = torch.full((n + PAD,), float("nan"), dtype=t.dtype, device=dev)
    elif t.dtype == torch.uint8:
        big = torch.full((n + PAD,), 0xFF, dtype=t.dtype, device=dev)
    else:
        big = torch.full((n + PAD,), 1 << 40, dtype=t.dtype, device=dev)
    off = 0 if where == "start" else PAD
    view = big[off:off + n].view(t.shape)
    view.copy_(t)
    return view, big


def run(bufs):
    e, p, w, bi, la, fl, ll, ws = bufs
    nll = torch.empty(B, device=dev)
    rc = lib.sc_rnnt_joint_fwd(ptr(e), ptr(p), ptr(w), ptr(bi), B, T, U, V, J, ptr(la), la.stride(0),
                               ptr(fl), ptr(ll), 0, ptr(nll), ptr(ws), wsb, stream_of(e))
    assert rc == 0, _lib.last_error() if hasattr(_lib, "last_error") else rc
    import ctypes
    geo = [ctypes.c_int(0) for _ in range(3)]
    lib.sc_rnnt_joint_geometry(B, T, U, V, *[ctypes.addressof(g) for g in geo])
    ntb, nus, S = (g.value for g in geo)
    scale = torch.ones(B, device=dev)
    d_enc = torch.empty(nus, B, T, J, device=dev)
    d_pred = torch.zeros(B, ntb, U + 1, J, device=dev)
    dW = torch.empty(S, V, J, device=dev)
    db = torch.empty(S, V, device=dev)
    rc = lib.sc_rnnt_joint_bwd(ptr(e), ptr(p), ptr(w), ptr(bi), B, T, U, V, J, ptr(la), la.stride(0),
                               ptr(fl), ptr(ll), 0, ptr(scale), ptr(d_enc), ptr(d_pred), ptr(dW),
                               ptr(db), ptr(ws), wsb, stream_of(e))
    assert rc == 0
    torch.cuda.synchronize()
    return [nll, d_enc.sum(0), d_pred.sum(1), dW.sum(0), db.sum(0)]


names = ["enc", "pred", "W", "bias", "labels", "flen", "llen", "ws"]
clean = [enc, pred, W, bias, labels, flen, llen, torch.zeros(wsb, dtype=torch.uint8, device=dev)]
ref = run(clean)
print("clean nll", ref[0].tolist())
for i, nm in enumerate(names):
    for where in ("start", "end"):
        bufs = list(clean)
        bufs[i], keep = embed(clean[i], where)
        out = run(bufs)
        diff = [k for k, (a, o) in enumerate(zip(ref, out)) if not torch.equal(a, o)]
        print(f"{nm:6s} {where:5s}: outputs differing {diff}"
              + (f" nll {out[0].tolist()}" if 0 in diff else ""), flush=True)
# ws garbage everywhere (uninitialised workspace)
ws = torch.full((wsb,), 0xFF, dtype=torch.uint8, device=dev)
out = run(clean[:7] + [ws])
print("ws all-0xFF:", [k for k, (a, o) in enumerate(zip(ref, out)) if not torch.equal(a, o)])
