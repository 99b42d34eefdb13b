#!/usr/bin/env python3
"""Time the fused RNN-T joiner kernels at the C5 lattice (B x T=1500 x U=150, V=1024, J=64):
forward (joint_fwd + rnnt_ab) and backward (joint_dz + joint_dw + partial sums), HIP events.
usage: python tools/joint_probe.py [B] [reps]   (run under rocprofv3 for per-kernel times)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from statecatcher_amd import ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    T, U, V, J = 1500, 150, 1024, 64
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    enc = (torch.randn(B, T, J, device=dev, generator=g) * 0.5).requires_grad_(True)
    pred = (torch.randn(B, U + 1, J, device=dev, generator=g) * 0.5).requires_grad_(True)
    W = (torch.randn(V, J, device=dev, generator=g) * 0.3).requires_grad_(True)
    bias = torch.zeros(V, device=dev, requires_grad=True)
    lab = torch.randint(1, V, (B, U), device=dev, generator=g)
    fl = torch.full((B,), T, dtype=torch.int64, device=dev)
    ll = torch.full((B,), U, dtype=torch.int64, device=dev)
    nodes = B * T * (U + 1)
    for r in range(reps + 1):
        e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        e0.record()
        nll = ops.RNNTJointFn.apply(enc, pred, W, bias, lab, fl, ll, 0)
        e1.record()
        nll.mean().backward()
        e2.record()
        torch.cuda.synchronize()
        if r:
            f, b = e0.elapsed_time(e1), e1.elapsed_time(e2)
            fl_f = nodes * V * J * 2
            print(f"B={B}: fwd {f:.2f} ms ({fl_f / f / 1e9:.0f} TFLOP/s logits), bwd {b:.2f} ms, "
                  f"{nodes / (f + b) / 1e3:.1f} M nodes/s", flush=True)


if __name__ == "__main__":
    main()
