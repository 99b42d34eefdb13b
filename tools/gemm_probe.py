#!/usr/bin/env python3
"""Time alternative formulations of the three LucyRNN GEMMs at the C2 shape (bf16, hipBLASLt
through torch) to pick the fastest layout.  usage: python tools/gemm_probe.py"""
import torch

M, Din, N = 48000, 512, 3584   # rows = B*T, layer input, 7*D
dev = "cuda"
x = torch.randn(M, Din, device=dev, dtype=torch.bfloat16)
w = torch.randn(N, Din, device=dev, dtype=torch.bfloat16)
b = torch.randn(N, device=dev, dtype=torch.bfloat16)
dg = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
wT = w.t().contiguous()


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
    print(f"{name:50s} {ms * 1e3:8.1f} us  {flops / ms / 1e9:8.1f} TF/s", flush=True)


F = 2 * M * N * Din
bench("fwd addmm(b, x, w.t())", lambda: torch.addmm(b, x, w.t()), F)
bench("fwd addmm(b, x, wT)", lambda: torch.addmm(b, x, wT), F)
bench("fwd x @ w.t()", lambda: x @ w.t(), F)
bench("dgrad dg @ w", lambda: dg @ w, F)
bench("dgrad dg @ wT.t()", lambda: dg @ wT.t(), F)
bench("dgrad (w.t() @ dg.t()).t()", lambda: (w.t() @ dg.t()).t(), F)
bench("dgrad (wT @ dg.t()).t()", lambda: (wT @ dg.t()).t(), F)
for S in (1, 4, 8, 16):
    def wg(S=S):
        if S == 1:
            return dg.t() @ x
        return torch.bmm(dg.view(S, M // S, N).transpose(1, 2), x.view(S, M // S, Din)).sum(0, dtype=torch.float32)
    bench(f"wgrad split-K {S}", wg, F)
    bench(f"wgrad x^T dg split-K {S} (transposed out)",
          (lambda S=S: (x.t() @ dg) if S == 1 else torch.bmm(x.view(S, M // S, Din).transpose(1, 2), dg.view(S, M // S, N)).sum(0, dtype=torch.float32)), F)
xo = torch.randn(M, 512, device=dev, dtype=torch.bfloat16)
wo = torch.randn(1024, 512, device=dev, dtype=torch.bfloat16)
bo = torch.randn(1024, device=dev, dtype=torch.bfloat16)
go = torch.randn(M, 1024, device=dev, dtype=torch.bfloat16)
Fo = 2 * M * 1024 * 512
bench("out fwd addmm", lambda: torch.addmm(bo, xo, wo.t()), Fo)
bench("out dgrad go @ wo", lambda: go @ wo, Fo)
bench("out wgrad split8", lambda: torch.bmm(go.view(8, M // 8, 1024).transpose(1, 2), xo.view(8, M // 8, 512)).sum(0, dtype=torch.float32), Fo)
x0 = torch.randn(M, 80, device=dev, dtype=torch.bfloat16)
w0 = torch.randn(N, 80, device=dev, dtype=torch.bfloat16)
F0 = 2 * M * N * 80
bench("layer0 fwd addmm (K=80)", lambda: torch.addmm(b, x0, w0.t()), F0)
bench("layer0 wgrad split8 (K=80)", lambda: torch.bmm(dg.view(8, M // 8, N).transpose(1, 2), x0.view(8, M // 8, 80)).sum(0, dtype=torch.float32), F0)
