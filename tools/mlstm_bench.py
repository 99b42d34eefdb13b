#!/usr/bin/env python3
"""mLSTM cell kernels (csrc/mlstm.hip) at the C4 bench shape: B = 32, NH = 4, T = 1536,
DQ = 96, DV = 192 (BH = 128), bf16 and f16.  HIP-event timing of sc_mlstm_fwd / sc_mlstm_bwd
over repeated launches, algorithmic bytes as ops.MLSTMFn counts them (fwd: q k v in, h out;
bwd: q k v h dh in, dq dk dv out).
usage: python tools/mlstm_bench.py [--bh 128] [--t 1536] [--reps 20]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from statecatcher_amd import _lib   # noqa: E402
from statecatcher_amd.ops import dtype_code, ptr   # noqa: E402


def arg(name, default):
    return int(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


BH, T, REPS = arg("--bh", 128), arg("--t", 1536), arg("--reps", 20)
DQ, DV, nc = 96, 192, T // 64
dev = "cuda"
lib = _lib.load()
st = torch.cuda.current_stream().cuda_stream


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(REPS):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


for cdt in (torch.bfloat16, torch.float16):
    g = torch.Generator(device=dev).manual_seed(0)
    q = torch.randn(BH, T, DQ, device=dev, generator=g).to(cdt)
    k = torch.randn(BH, T, DQ, device=dev, generator=g).to(cdt)
    v = torch.randn(BH, T, DV, device=dev, generator=g).to(cdt)
    ig = torch.randn(BH, T, device=dev, generator=g) * 3
    fg = torch.randn(BH, T, device=dev, generator=g) * 2 + 3
    h = torch.empty(BH, T, DV, dtype=cdt, device=dev)
    Cs = torch.empty(BH, nc, DQ, DV, dtype=cdt, device=dev)
    cT = torch.empty(BH, DQ, DV, device=dev)
    ns = torch.empty(BH, nc + 1, DQ, device=dev)
    ms = torch.empty(BH, nc + 1, device=dev)
    mrow = torch.empty(BH, T, device=dev)
    den = torch.empty(BH, T, device=dev)
    dh = torch.randn(BH, T, DV, device=dev, generator=g).to(cdt)
    dC0 = torch.empty(BH, DQ, DV, device=dev)
    dn0 = torch.empty(BH, DQ, device=dev)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    qdq = torch.empty(BH, T, device=dev)
    kdk = torch.empty(BH, T, device=dev)
    dc = dtype_code(q)

    def fwd():
        rc = lib.sc_mlstm_fwd(ptr(q), ptr(k), ptr(v), dc, ptr(ig), ptr(fg), None, None, None, BH,
                              T, DQ, DV, 1e-6, ptr(h), ptr(Cs), ptr(ns), ptr(ms), ptr(cT),
                              ptr(mrow), ptr(den), None, st)
        assert rc == 0

    def bwd():
        rc = lib.sc_mlstm_bwd(ptr(q), ptr(k), ptr(v), dc, ptr(ig), ptr(fg), ptr(h), ptr(dh), None,
                              None, ptr(Cs), ptr(ns), ptr(ms), ptr(mrow), ptr(den), BH, T, DQ, DV,
                              1e-6, ptr(dC0), ptr(dn0), ptr(dq), ptr(dk), ptr(dv), ptr(qdq),
                              ptr(kdk), None, st)
        assert rc == 0

    tf, tb = timeit(fwd), timeit(bwd)
    fb = BH * T * (2 * DQ + 2 * DV) * 2
    bb = BH * T * (4 * DQ + 4 * DV) * 2
    print(f"{str(cdt):15s} BH={BH} T={T}: fwd {tf:7.1f} us ({fb / tf / 1e3:6.0f} GB/s, "
          f"{tf / nc:5.2f} us/chunk) | bwd {tb:7.1f} us ({bb / tb / 1e3:6.0f} GB/s, "
          f"{tb / nc:5.2f} us/chunk)", flush=True)
