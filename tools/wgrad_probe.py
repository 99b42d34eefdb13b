#!/usr/bin/env python3
"""Weight-gradient GEMM formulations at the C2 shape with PyTorch TunableOp tuning ON for each
(so every variant is timed with its best hipBLASLt/rocBLAS solution, not the heuristic pick).
dW [3584, 512] fp32 = dG[48000, 3584]^T X[48000, 512], bf16 inputs.
usage: python tools/wgrad_probe.py [tuned_out.csv]"""
import os
import sys

import torch
import torch.cuda.tunable as tun

out_csv = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wgrad_tuned.csv"
tun.enable(True)
tun.tuning_enable(True)
tun.set_max_tuning_duration(150)
tun.set_filename(out_csv)

M, K, N = 48000, 512, 3584
dev = "cuda"
torch.manual_seed(0)
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
dg = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
ref = (dg.float().t() @ x.float())
F = 2 * M * N * K


def bench(name, fn, it=20):
    y = fn()
    torch.cuda.synchronize()
    err = float((y.float() - ref).abs().max() / ref.abs().max())
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(f"{name:55s} {ms * 1e3:8.1f} us  {F / ms / 1e9:7.1f} TF/s  relerr {err:.1e}", flush=True)


def splitk(S, trans=False):
    if trans:   # x^T dG per slice -> [S, K, N], summed, transposed view
        return lambda: torch.bmm(x.view(S, M // S, K).transpose(1, 2),
                                 dg.view(S, M // S, N)).sum(0, dtype=torch.float32).t()
    return lambda: torch.bmm(dg.view(S, M // S, N).transpose(1, 2),
                             x.view(S, M // S, K)).sum(0, dtype=torch.float32)


bench("mm dG^T X (bf16 out)", lambda: dg.t() @ x)
bench("mm X^T dG (bf16 out) .t()", lambda: (x.t() @ dg).t())
if hasattr(torch, "mm") and "out_dtype" in (torch.mm.__doc__ or ""):
    bench("mm dG^T X out_dtype=fp32", lambda: torch.mm(dg.t(), x, out_dtype=torch.float32))
for S in (4, 8, 16, 24, 32):
    bench(f"bmm split-K {S} dG^T X + fp32 sum", splitk(S))
    bench(f"bmm split-K {S} X^T dG + fp32 sum (.t())", splitk(S, True))
tun.write_file() if hasattr(tun, "write_file") else None
print("tuned entries ->", out_csv, os.path.exists(out_csv))
