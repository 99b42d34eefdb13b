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


def timeit(fn, iters, rounds=5):
    """min over `rounds` of the mean launch time of `iters` back-to-back calls; fn(i) should
    rotate its inputs over buffers larger than the 256 MB Infinity Cache (single-buffer
    repeats of a ~400 MB stream time unreliably, tools/scan_probe.hip)."""
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / iters * 1e-3)
    return best


def report(name, sec, nbytes):
    print(f"{name:28s} {sec * 1e6:9.1f} us  {nbytes / sec / 1e9:8.1f} GB/s  "
          f"{nbytes / sec / 8e12 * 100:5.1f}% of 8 TB/s", flush=True)


e = torch.finfo(dt).bits // 8
NROT = 4
if args.only in ("all", "scan"):
    bias = torch.randn(7, D, device=dev) * 0.1
    h0 = torch.zeros(B, D, device=dev)
    s0 = torch.zeros(B, D, device=dev)
    dout = [torch.randn(B, T, D, device=dev).to(dt) for _ in range(NROT)]
    for lay in ["plain", "blocked"]:
        gs = []
        for _ in range(NROT):
            g = (torch.randn(B, T, 7, D, device=dev) * 0.5).to(dt)
            gs.append(g if lay == "plain" else g.view(B, T, 7, D // 64, 64).permute(0, 1, 3, 2, 4).contiguous())
        fw = [ops._scan_fwd(g, h0, s0, True, bias) for g in gs]
        ck = fw[0][3]
        nb_f = B * T * D * 8 * e + ck.numel() * 4
        report(f"lucy_scan_fwd {args.dtype} {lay}",
               timeit(lambda i: ops._scan_fwd(gs[i % NROT], h0, s0, True, bias), args.iters), nb_f)
        nb_b = B * T * D * 15 * e + ck.numel() * 4
        report(f"lucy_scan_bwd {args.dtype} {lay}",
               timeit(lambda i: ops._scan_bwd(gs[i % NROT], fw[i % NROT][3], dout[i % NROT], None, True,
                                              bias), args.iters), nb_b)
        del gs, fw
if args.only in ("all", "ln"):
    x = torch.randn(B * T, D, device=dev).to(dt)
    gam = torch.ones(D, device=dev, requires_grad=True)
    bet = torch.zeros(D, device=dev, requires_grad=True)
    report("layernorm_fwd", timeit(lambda i: ops.layer_norm(x, gam, bet), args.iters), 2 * B * T * D * e)
if args.only in ("all", "ctc"):
    logits = (torch.randn(B, T, V, device=dev) * 2).to(dt)
    tl = torch.randint(50, 151, (B,), device=dev)
    tg = torch.randint(1, V, (B, 150), device=dev)
    il = torch.full((B,), T, device=dev, dtype=torch.int64)
    report("ctc_fwd (emit+chain+ab)", timeit(lambda i: ops.ctc_nll(logits, tg, il, tl), args.iters),
           B * T * V * e)
    lg = logits.clone().requires_grad_(True)

    def fb(i):
        lg.grad = None
        ops.ctc_nll(lg, tg, il, tl).sum().backward()
    report("ctc_fwd+bwd", timeit(fb, args.iters), 2 * B * T * V * e)
if args.only in ("all", "rnnt"):
    # config C5's lattice per sequence (T=1500, U=150, V=1024) at B=4: 1.86 GB of bf16 logits
    Br, Tr, Ur = 4, 1500, 150
    lg = (torch.randn(Br, Tr, Ur + 1, V, device=dev) * 2).to(dt)
    lab = torch.randint(1, V, (Br, Ur), device=dev)
    fl = torch.full((Br,), Tr, device=dev, dtype=torch.int64)
    ll = torch.full((Br,), Ur, device=dev, dtype=torch.int64)
    nb = Br * Tr * (Ur + 1) * V * e
    report("rnnt fwd (emit+lattice)", timeit(lambda i: ops.rnnt_loss(lg, lab, fl, ll, is_logits=True),
                                             max(3, args.iters // 4)), nb)
    lgr = lg.clone().requires_grad_(True)

    def rb(i):
        lgr.grad = None
        ops.rnnt_loss(lgr, lab, fl, ll, is_logits=True).backward()
    report("rnnt fwd+bwd", timeit(rb, max(3, args.iters // 4)), 3 * nb)
if args.only in ("all", "mlstm"):
    # config C4's cell: d=768, 4 heads (DQ 96, DV 192), T=1536 (1500 padded to 64), B=32
    Bm, NHm, Tm, DQm, DVm = 32, 4, 1536, 96, 192
    qm = torch.randn(Bm, NHm, Tm, DQm, device=dev, dtype=torch.bfloat16)
    km = torch.randn(Bm, NHm, Tm, DQm, device=dev, dtype=torch.bfloat16)
    vm = torch.randn(Bm, NHm, Tm, DVm, device=dev, dtype=torch.bfloat16)
    igm = torch.randn(Bm, NHm, Tm, device=dev) * 3
    fgm = torch.randn(Bm, NHm, Tm, device=dev) * 2 + 3
    nc = Tm // 64
    io = Bm * NHm * Tm * (2 * DQm + 2 * DVm) * 2
    st_bytes = Bm * NHm * (nc + 1) * DQm * DVm * 4
    report("mlstm fwd (C pass + H pass)", timeit(lambda i: ops.mlstm_chunkwise(qm, km, vm, igm, fgm),
                                                 args.iters), io + 2 * st_bytes)
    qg, kg, vg = (x.clone().requires_grad_(True) for x in (qm, km, vm))

    def mb(i):
        qg.grad = kg.grad = vg.grad = None
        ops.mlstm_chunkwise(qg, kg, vg, igm, fgm).float().sum().backward()
    report("mlstm fwd+bwd", timeit(mb, args.iters), 3 * io + 6 * st_bytes)
if args.only in ("all", "fbank"):
    # one C2 batch of audio: 32 x 15 s at 16 kHz -> 1500 frames per row (make_frontend, mfcc)
    ns = (T - 1) * 160 + 400
    audio = [torch.randn(B, ns, device=dev) * 0.3 for _ in range(2)]
    for kind in ("mfcc", "mel"):
        sec = timeit(lambda i: ops.fbank(audio[i % 2], kind), args.iters)
        # FLOPs per frame: two 20-point DFT stages (20 x 400 real MACs + 20 x 201 complex MACs),
        # twiddles, mel bands (~2 x 201 MACs) and, for mfcc, the 80 x 80 DCT
        flops = 2 * (20 * 400 * 2 + 20 * 201 * 4 + 400 * 4 + 402) + (2 * 80 * 80 if kind == "mfcc" else 0)
        print(f"fbank_{kind:4s} {sec * 1e6:9.1f} us  {B * T / sec / 1e6:8.2f} M frames/s  "
              f"{B * T * flops / sec / 1e12:6.2f} TFLOP/s fp32  "
              f"({B * T / sec / 100:.0f}x realtime of one 100-fps stream)", flush=True)
