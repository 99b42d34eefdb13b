#!/usr/bin/env python3
"""Weight-gradient GEMM at the C2 shapes: the MFMA split-L kernel (gemm.hip + slab sum) against
the hipBLASLt split-K path (TunableOp table on), HIP-event timing over rotating inputs.
usage: python tools/gemm_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from statecatcher_amd import ops, _lib  # noqa: E402

tab = os.path.join(ROOT, "statecatcher_amd", "tuning", "tunableop_gfx950.csv")
if os.path.exists(tab):
    import torch.cuda.tunable as tun
    tun.enable(True)
    tun.tuning_enable(False)
    tun.read_file(tab)

dev = "cuda"
lib = _lib.load()


def timeit(fn, n=20):
    for _ in range(3):
        fn(0)
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(n):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return best


QUICK = "--quick" in sys.argv   # gate shape only, no library baseline
for (L, I, J, blk) in [(48000, 3584, 512, 512), (48000, 1024, 512, 0)][:1 if QUICK else 2]:
    R = 3
    dys = [torch.randn(L, I, device=dev).to(torch.bfloat16) for _ in range(R)]
    xs = [torch.randn(L, J, device=dev).to(torch.bfloat16) for _ in range(R)]
    F = 2.0 * L * I * J
    S = lib.sc_gemm_wgrad_splits(L, I, J)
    part = torch.empty(S, I, J, dtype=torch.float32, device=dev)

    def kern_only(i):
        lib.sc_gemm_wgrad_bf16(_lib.ptr(dys[i % R]), I, _lib.ptr(xs[i % R]), J, _lib.ptr(part),
                               L, I, J, S, _lib.stream_of(part))

    t_k = timeit(kern_only)
    t_m = timeit(lambda i: ops.wgrad_mfma(dys[i % R], xs[i % R], blk))
    os.environ["SC_NO_MFMA_WGRAD"] = "1"

    def lib_path(i):
        M, N = dys[i % R].shape
        return ops.wgrad_splitk.__wrapped__(dys[i % R], xs[i % R], blk) \
            if hasattr(ops.wgrad_splitk, "__wrapped__") else None

    # the hipBLASLt formulation wgrad_splitk used before the MFMA kernel (S=16 batched + sum)
    def blas(i):
        dy, x = dys[i % R], xs[i % R]
        Sb = 16
        p = torch.bmm(dy.view(Sb, L // Sb, I).transpose(1, 2), x.view(Sb, L // Sb, J))
        return ops.colsum(p.view(Sb, I * J), (blk // 64, 7) if blk else (1, 1))

    t_b = timeit(blas) if not QUICK else float("nan")
    ref = dys[0].float().t() @ xs[0].float()
    got = ops.wgrad_mfma(dys[0], xs[0], 0)
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    print(f"L={L} I={I} J={J} S={S}: mfma kernel {t_k:7.1f} us ({F / t_k / 1e6:6.1f} TF/s), "
          f"+slab sum {t_m:7.1f} us ({F / t_m / 1e6:6.1f} TF/s) | hipBLASLt split-K 16 + sum "
          f"{t_b:7.1f} us ({F / t_b / 1e6:6.1f} TF/s) | relerr {err:.1e}", flush=True)
