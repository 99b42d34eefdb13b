#!/usr/bin/env python3
"""Frame-major projection GEMMs at the C2 shapes: the persistent MFMA kernel (tn_gemm.hip)
against the library GEMM torch.matmul picks (TunableOp table on), interleaved rounds in one
process, HIP-event timing over rotating random inputs.
usage: python tools/tn_bench.py [--tm 128|192|256|257]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from statecatcher_amd import ops  # noqa: E402

tab = os.path.join(ROOT, "statecatcher_amd", "tuning", "tunableop_gfx950.csv")
if os.path.exists(tab):
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(tab)

dev = "cuda"
TMS = [int(sys.argv[sys.argv.index("--tm") + 1])] if "--tm" in sys.argv else [257, 256]


def timeit(fn, n=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


SHAPES = [("gate fwd", 48000, 3584, 512), ("layer-0 fwd", 48000, 3584, 128),
          ("gate dgrad", 48000, 512, 3584), ("out-proj dgrad", 48000, 512, 1024),
          ("out-proj fwd", 48000, 1024, 512)]
if "--shapes" in sys.argv:   # e.g. --shapes 0,2: a subset of SHAPES by index
    SHAPES = [SHAPES[int(i)] for i in sys.argv[sys.argv.index("--shapes") + 1].split(",")]
NOLIB = "--nolib" in sys.argv
LN = "--ln" in sys.argv   # the LayerNorm-fold GEMM (sc_gemm_tn_ln_bf16) against the plain library GEMM
for name, M, N, K in SHAPES:
    R = 3
    As = [torch.randn(M, K, device=dev).to(torch.bfloat16) for _ in range(R)]
    Bs = [torch.randn(N, K, device=dev).to(torch.bfloat16) for _ in range(R)]
    F = 2.0 * M * N * K
    if LN:
        rv = torch.randn(N, device=dev) * 0.01
        arms = {"ln": lambda i: ops.gemm_tn_ln(As[i % R], Bs[i % R], rv, 1e-5)}
    else:
        arms = {f"tn{tm}": (lambda tm: lambda i: ops.gemm_tn(As[i % R], Bs[i % R], tm))(tm) for tm in TMS}
    arms["lib"] = lambda i: torch.matmul(As[i % R], Bs[i % R].t())
    Bts = [b.t().contiguous() for b in Bs]
    if not NOLIB:
        arms["libNN"] = lambda i: torch.matmul(As[i % R], Bts[i % R])
    for f in arms.values():   # warm-up
        for i in range(3):
            f(i)
    torch.cuda.synchronize()
    res = {k: [] for k in arms}
    for _ in range(5):
        for k, f in arms.items():
            res[k].append(timeit(f))
    ref = As[0].float() @ Bs[0].float().t()
    if LN:   # rstd (h W^T - mean r) with the rows' own statistics
        h = As[0].float()
        mu, var = h.mean(1, keepdim=True), h.var(1, unbiased=False, keepdim=True)
        ref = (ref - mu * rv[None, :]) * torch.rsqrt(var + 1e-5)
        got = ops.gemm_tn_ln(As[0], Bs[0], rv, 1e-5)[0]
    else:
        got = ops.gemm_tn(As[0], Bs[0], TMS[0])
    err = ((got.float() - ref).abs().max() / ref.abs().max()).item()
    line = " | ".join(f"{k} med {sorted(v)[2]:6.1f} min {min(v):6.1f} us "
                      f"({F / sorted(v)[2] / 1e6:6.1f} TF/s)" for k, v in res.items())
    out_gbs = M * N * 2 / (min(res["ln" if LN else f"tn{TMS[0]}"]) * 1e-6) / 1e9
    del Bts
    print(f"{name:15s} M={M} N={N} K={K}: {line} | relerr {err:.1e} | C write {out_gbs:.0f} GB/s",
          flush=True)
    del As, Bs
