"""A/B of the xLSTM projection weight-gradient tail (N = 2312 at C4: rows 2304..2311) in one
process: the library M=8 GEMM vs the MFMA kernel over the last 256-row window."""
import torch
from statecatcher_amd import ops

dev = torch.device("cuda:0")
L, N, K = 48000, 2312, 768
dy = torch.randn(L, N, device=dev).to(torch.bfloat16)
x = torch.randn(L, K, device=dev).to(torch.bfloat16)
n0 = N - N % 256


def lib_tail():
    return ops._mm_f32(dy[:, n0:].t(), x)


def win_tail():
    return ops.wgrad_mfma(dy[:, N - 256:], x)[256 - (N - n0):]


for f in (lib_tail, win_tail):
    for _ in range(3):
        f()
torch.cuda.synchronize()
ref = dy[:, n0:].float().t() @ x.float()
for name, f in (("library M=8", lib_tail), ("MFMA window", win_tail), ("library M=8", lib_tail),
                ("MFMA window", win_tail)):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        out = f()
    e1.record()
    torch.cuda.synchronize()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f"{name}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us  rel err {err:.2e}", flush=True)
