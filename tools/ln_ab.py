"""LayerNorm forward A/B (GPU): outputs (y, and the saved mean / rstd through a backward) of
ops.layer_norm with the library this process loads (SC_LIB_PATH), saved; `compare` checks two
saves bitwise.  usage: python tools/ln_ab.py save out.pt | compare a.pt b.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if sys.argv[1] == "save":
    from statecatcher_amd import ops
    out = {}
    for dt in (torch.bfloat16, torch.float32):
        for rows, D in ((48000, 512), (4097, 512), (3, 1024), (12345, 1024)):
            g = torch.Generator().manual_seed(rows + D)
            x = (torch.randn(rows, D, generator=g) * 2 + 0.5).to(dt).cuda().requires_grad_()
            gam = (torch.rand(D, generator=g) + 0.5).cuda().requires_grad_()
            bet = torch.randn(D, generator=g).cuda().requires_grad_()
            y = ops.layer_norm(x, gam, bet)
            dy = torch.randn(rows, D, generator=g).to(dt).cuda()
            y.backward(dy)
            k = f"{str(dt)[6:]}_{rows}_{D}"
            out[k + "_y"] = y.detach().float().cpu()
            out[k + "_dx"] = x.grad.float().cpu()
            out[k + "_dg"] = gam.grad.cpu()
            out[k + "_db"] = bet.grad.cpu()
    torch.cuda.synchronize()
    torch.save(out, sys.argv[2])
    print("saved", len(out))
else:
    a = torch.load(sys.argv[2], weights_only=True)
    b = torch.load(sys.argv[3], weights_only=True)
    bad = [k for k in a if not torch.equal(a[k], b[k])]
    print(f"{len(a)} tensors, {len(bad)} differ: {bad[:8]}")
    sys.exit(1 if bad else 0)
