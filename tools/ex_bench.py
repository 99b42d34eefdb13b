"""Emission-logit GEMM variants (tool): the [B, T, U + 1] exact emission columns of the bf16 C2
head (ops._emission_logits) as one batched GEMM, timed with HIP events, several orientations /
paddings.  python tools/ex_bench.py"""
import torch

B, T, D, U1, V = 32, 1500, 512, 151, 1024
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
wide = torch.randn(B, T, 3 * D, device=dev, generator=g).to(torch.bfloat16)
img = torch.randn(V, 3 * D, device=dev, generator=g).to(torch.bfloat16)
lab = torch.randint(0, V, (B, U1), device=dev, generator=g)


def timeit(f, n=20):
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def v_cur():
    wg = img[lab]
    return torch.bmm(wide, wg.transpose(1, 2), out_dtype=torch.float32)


def v_trans():
    wg = img[lab]
    return torch.bmm(wg, wide.transpose(1, 2), out_dtype=torch.float32)


def v_pad(n):
    labp = torch.cat([lab, lab[:, :n - U1]], 1)
    def f():
        wg = img[labp]
        return torch.bmm(wide, wg.transpose(1, 2), out_dtype=torch.float32)
    return f


def v_full():   # every column: one [B*T, 3D] x [3D, V] GEMM
    return torch.mm(wide.view(-1, 3 * D), img.t(), out_dtype=torch.float32)


ref = v_cur()
assert torch.allclose(v_trans().transpose(1, 2), ref)
for name, f in (("current [B,T,3D]x[B,3D,U1]", v_cur), ("transposed [B,U1,3D]x[B,3D,T]", v_trans),
                ("padded U1->160", v_pad(160)), ("padded U1->192", v_pad(192)),
                ("padded U1->256", v_pad(256)), ("full split GEMM (all V)", v_full)):
    print(f"{name:36s} {timeit(f):8.1f} us")
