#!/usr/bin/env python3
"""Debug helper: fused joiner gradients vs the fp64 restatement of tests/test_gpu_rnnt_joint.py,
per gradient and per frame.  usage: python tools/joint_debug.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import test_gpu_rnnt_joint as t  # noqa: E402

DEV = torch.device("cuda:0")
for (B, T, Umax, V, Tb, Ub) in [(1, 37, 0, 64, None, None), (1, 37, 1, 64, None, None),
                                (1, 37, 3, 64, None, None), (1, 32, 3, 64, None, None),
                                (1, 37, 3, 1024, None, None), (3, 37, 7, 64, [37, 20, 33], [7, 3, 0])]:
    joiner, enc_out, labels, fl, ll = t.case(B, T, Umax, V, B * 100 + T, Tb, Ub)
    joiner = joiner.to(DEV)
    prefix = torch.cat([torch.zeros(B, 1, dtype=torch.long), labels], 1).to(DEV)
    enc_p, pred_p, W, bias = joiner(enc_out.to(DEV), prefix, project_only=True)
    enc_p, pred_p, W, bias = (x.detach().requires_grad_(True) for x in (enc_p, pred_p, W, bias))
    nll = t.sc().ops.RNNTJointFn.apply(enc_p, pred_p, W, bias, labels.to(DEV), fl.to(DEV), ll.to(DEV), 0)
    nll.mean().backward()
    rn, ge, gp, gw, gb = t.ref_fp64(enc_p.detach(), pred_p.detach(), W.detach(), bias.detach(),
                                    labels, fl, ll, 0)
    errs = {n: round(t.rel(g, r), 4) for n, g, r in [("enc", enc_p.grad, ge), ("pred", pred_p.grad, gp),
                                                    ("W", W.grad, gw), ("bias", bias.grad, gb)]}
    d = (enc_p.grad[0].double().cpu() - ge[0]).norm(dim=-1) / ge[0].norm(dim=-1).clamp_min(1e-30)
    print(B, T, Umax, V, errs, "enc rel per t (b=0):", [round(float(x), 3) for x in d[:40]], flush=True)
