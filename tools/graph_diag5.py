"""Diagnostic (GPU): the RNN-T joint forward alone under graph capture: (a) the raw C call on
eager buffers, (b) RNNTJointFn on eager fp32 inputs, (c) on bf16 inputs; each replayed after the
eager pool is filled with NaN tensors."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from statecatcher_amd import _lib, ops  # noqa: E402
from statecatcher_amd._lib import ptr, stream_of  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
B, T, U, V, J = 2, 200, 12, 256, 64
enc = torch.randn(B, T, J, device=dev) * 0.5
pred = torch.randn(B, U + 1, J, device=dev) * 0.5
W = torch.randn(V, J, device=dev) * 0.1
bias = torch.randn(V, device=dev) * 0.1
lens = torch.tensor([12, 7], device=dev)
labels = torch.randint(1, V, (B, U), device=dev)
for b in range(B):
    labels[b, lens[b]:] = 0
flen = torch.full((B,), T, device=dev, dtype=torch.int64)
llen = lens.to(torch.int64)
lib = _lib.load()
wsb = lib.sc_rnnt_workspace_bytes(B, T, U)
Wb = W.to(torch.bfloat16)
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
nll = torch.empty(B, device=dev)


def raw():
    rc = lib.sc_rnnt_joint_fwd(ptr(enc), ptr(pred), ptr(Wb), ptr(bias), B, T, U, V, J, ptr(labels),
                               labels.stride(0), ptr(flen), ptr(llen), 0, ptr(nll), ptr(ws), wsb,
                               stream_of(enc))
    assert rc == 0
    return nll


def fn32():
    return ops.RNNTJointFn.apply(enc, pred, W, bias, labels, flen, llen, 0)


encb, predb = enc.to(torch.bfloat16), pred.to(torch.bfloat16)


def fn16():
    return ops.RNNTJointFn.apply(encb, predb, W, bias, labels, flen, llen, 0)


for name, f in (("raw", raw), ("fn32", fn32), ("fn16", fn16)):
    ref = f().clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        f()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = f()
    torch.cuda.synchronize()
    for poison in (False, True, False):
        keep = [torch.full((2 ** k,), float("nan"), device=dev) for k in range(4, 27)] * 2 \
            if poison else []
        g.replay()
        torch.cuda.synchronize()
        print(f"{name} poison {poison}: equal {torch.equal(ref, out)} ref {ref.tolist()} "
              f"out {out.tolist()}", flush=True)
        del keep
