#!/usr/bin/env python3
"""Compare hipBLASLt vs rocBLAS (torch preferred_blas_library) and TunableOp for the LucyRNN
GEMMs at the C2 shape.  usage: python tools/blas_probe.py [tune]"""
import os
import sys

import torch

M, Din, N = 48000, 512, 3584
dev = "cuda"
torch.manual_seed(0)
x = torch.randn(M, Din, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, Din, device=dev, dtype=torch.bfloat16)
b = torch.randn(N, device=dev, dtype=torch.bfloat16)
dg = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
S = 16
dgS = dg.view(S, M // S, N).transpose(1, 2)
xS = x.view(S, M // S, Din)
x0 = torch.randn(M, 80, device=dev, dtype=torch.bfloat16)
w0 = torch.randn(N, 80, device=dev, dtype=torch.bfloat16)
xo = torch.randn(M, 512, device=dev, dtype=torch.bfloat16)
wo = torch.randn(1024, 512, device=dev, dtype=torch.bfloat16)
bo = torch.randn(1024, device=dev, dtype=torch.bfloat16)
go = torch.randn(M, 1024, device=dev, dtype=torch.bfloat16)


def bench(name, fn, flops, it=20):
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
    print(f"  {name:40s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:8.1f} TF/s", flush=True)


F = 2 * M * N * Din
cases = [
    ("fwd addmm(b,x,w.t())", lambda: torch.addmm(b, x, w.t()), F),
    ("fwd x@w.t() (no bias)", lambda: x @ w.t(), F),
    ("dgrad dg@w", lambda: dg @ w, F),
    ("wgrad bmm split16", lambda: torch.bmm(dgS, xS), F),
    ("l0 fwd addmm K=80", lambda: torch.addmm(b, x0, w0.t()), 2 * M * N * 80),
    ("l0 wgrad bmm split16 K=80", lambda: torch.bmm(dgS, x0.view(S, M // S, 80)), 2 * M * N * 80),
    ("out fwd addmm", lambda: torch.addmm(bo, xo, wo.t()), 2 * M * 1024 * 512),
    ("out dgrad", lambda: go @ wo, 2 * M * 1024 * 512),
    ("out wgrad bmm split16", lambda: torch.bmm(go.view(S, M // S, 1024).transpose(1, 2), xo.view(S, M // S, 512)), 2 * M * 1024 * 512),
]
if len(sys.argv) > 1 and sys.argv[1] == "tune":
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_filename(os.path.join(os.environ.get("OUT", "."), "tunableop_results%d.csv"))
    print("TunableOp tuning:", flush=True)
    for name, fn, fl in cases:
        bench(name, fn, fl)
    torch.cuda.tunable.write_file()
else:
    for lib in ["cublaslt", "cublas"]:
        torch.backends.cuda.preferred_blas_library(lib)
        print("backend", lib, torch.backends.cuda.preferred_blas_library(), flush=True)
        for name, fn, fl in cases:
            bench(name, fn, fl)
