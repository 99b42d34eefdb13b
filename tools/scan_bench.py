#!/usr/bin/env python3
"""Standalone timing of the HIP hot-path kernels at the C2 shape (B=32, T=1500, D=512, V=1024)
with HIP events, interleaving repetitions in one process.  Prints achieved GB/s against the
algorithmic bytes of SURVEY §8(d).  usage: python tools/scan_bench.py [--iters N] [--only scan]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from statecatcher_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--only", default="all")
ap.add_argument("--dtype", default="bf16")
args = ap.parse_args()
dt = {"bf16": torch.bfloat16, "fp32": torch.float32, "fp16": torch.float16}[args.dtype]
dev = "cuda"
B, T, D, V = 32, 1500, 512, 1024
torch.manual_seed(0)


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def report(name, sec, nbytes):
    print(f"{name:28s} {sec * 1e6:9.1f} us  {nbytes / sec / 1e9:8.1f} GB/s  "
          f"{nbytes / sec / 8e12 * 100:5.1f}% of 8 TB/s", flush=True)


e = torch.finfo(dt).bits // 8
if args.only in ("all", "scan"):
    gates = (torch.randn(B, T, 7, D, device=dev) * 0.5).to(dt)
    bias = torch.randn(7, D, device=dev) * 0.1
    h0 = torch.zeros(B, D, device=dev)
    s0 = torch.zeros(B, D, device=dev)
    g, out, s_out, ckpt = ops._scan_fwd(gates, h0, s0, True, bias)
    nb_f = B * T * D * 8 * e + ckpt.numel() * 4
    report(f"lucy_scan_fwd {args.dtype}", timeit(lambda: ops._scan_fwd(gates, h0, s0, True, bias), args.iters), nb_f)
    dout = torch.randn(B, T, D, device=dev).to(dt)
    nb_b = B * T * D * 15 * e + ckpt.numel() * 4
    report(f"lucy_scan_bwd {args.dtype}",
           timeit(lambda: ops._scan_bwd(g, ckpt, dout, None, True, bias), args.iters), nb_b)
if args.only in ("all", "ln"):
    x = torch.randn(B * T, D, device=dev).to(dt)
    gam = torch.ones(D, device=dev, requires_grad=True)
    bet = torch.zeros(D, device=dev, requires_grad=True)
    report("layernorm_fwd", timeit(lambda: ops.layer_norm(x, gam, bet), args.iters), 2 * B * T * D * e)
if args.only in ("all", "ctc"):
    logits = (torch.randn(B, T, V, device=dev) * 2).to(dt)
    tl = torch.randint(50, 151, (B,), device=dev)
    tg = torch.randint(1, V, (B, 150), device=dev)
    il = torch.full((B,), T, device=dev, dtype=torch.int64)
    report("ctc_fwd (emit+chain+ab)", timeit(lambda: ops.ctc_nll(logits, tg, il, tl), args.iters),
           B * T * V * e)
    lg = logits.clone().requires_grad_(True)

    def fb():
        lg.grad = None
        ops.ctc_nll(lg, tg, il, tl).sum().backward()
    report("ctc_fwd+bwd", timeit(fb, args.iters), 2 * B * T * V * e)
