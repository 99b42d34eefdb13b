"""CTC gradient A/B (GPU): the loss and gradients of a set of CTC cases with the library this
process loads (SC_LIB_PATH), saved to a file; `compare` checks two such files bitwise.
  python tools/ctc_grad_ab.py save out.pt
  python tools/ctc_grad_ab.py compare a.pt b.pt
Cases: raw logits (bf16 / fp32; ragged lengths, labels from a small alphabet so repeats and
chains occur, a block of -inf vocabulary columns), and whole-model steps through compute_loss
under bf16 autocast (the exact split head: the emission columns from the fp32 side array) at a
small size and at C2's (6 x 512, V 1024, T 1500)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cases():
    from statecatcher_amd import ops
    from statecatcher_amd.model import ASRModel, CTCLoss, build_lucyrnn_config, compute_loss
    dev = torch.device("cuda")
    out = {}
    for dt in (torch.bfloat16, torch.float32):
        for ninf in (False, True):
            g = torch.Generator().manual_seed(3)
            B, T, V, U = 6, 400, 1024, 120
            x = (torch.randn(B, T, V, generator=g) * 3).to(dt)
            if ninf:
                x[:, :, 600:640] = -float("inf")
            x = x.to(dev).requires_grad_()
            tl = torch.randint(U // 3, U + 1, (B,), generator=g)
            il = torch.randint(T // 2, T + 1, (B,), generator=g)
            il[0] = T
            tg = torch.randint(1, 24, (B, U), generator=g)
            for b in range(B):
                tg[b, tl[b]:] = 0
            loss = ops.ctc_loss(x, tg.to(dev), il.to(dev), tl.to(dev), blank=0)
            loss.backward()
            key = f"logits_{str(dt)[6:]}_{'ninf' if ninf else 'plain'}"
            out[key + "_loss"] = loss.detach().float().cpu()
            out[key + "_grad"] = x.grad.float().cpu()
    for name, (L, H, V, B, T, U) in {"small": (3, 256, 256, 4, 300, 40),
                                     "c2": (6, 512, 1024, 2, 1500, 150)}.items():
        torch.manual_seed(5)
        model = ASRModel(None, build_lucyrnn_config(80, H, L, V), vocab_size=V, feat_dim=80,
                         proj_dim=-1).to(dev)
        with torch.no_grad():
            model.encoder.output_proj.weight.normal_(0, 0.02)
        g = torch.Generator().manual_seed(6)
        feats = torch.randn(B, T, 80, generator=g).to(dev)
        tl = torch.randint(U // 2, U + 1, (B,), generator=g)
        tg = torch.randint(1, V, (B, U), generator=g)
        for b in range(B):
            tg[b, tl[b]:] = 0
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss, _, _, _ = compute_loss("ctc", CTCLoss(blank=0, zero_infinity=True), model, feats,
                                         torch.ones(B, T, dtype=torch.bool, device=dev), tg.to(dev),
                                         torch.full((B,), T, device=dev), tl.to(dev), 0)
        loss.backward()
        out[f"model_{name}_loss"] = loss.detach().float().cpu()
        for n, p in model.named_parameters():
            out[f"model_{name}_{n}"] = p.grad.detach().float().cpu()
    torch.cuda.synchronize()
    return out


if __name__ == "__main__":
    if sys.argv[1] == "save":
        torch.save(cases(), sys.argv[2])
        print("saved", sys.argv[2])
    else:
        a = torch.load(sys.argv[2], weights_only=True)
        b = torch.load(sys.argv[3], weights_only=True)
        # (NaN where both have NaN counts as equal: -inf logits give NaN gradients in both)
        bad = [k for k in a if not (a[k].shape == b[k].shape and torch.equal(a[k].isnan(), b[k].isnan())
                                    and torch.equal(a[k].nan_to_num(0.0), b[k].nan_to_num(0.0)))]
        print(f"{len(a)} tensors, {len(bad)} differ: {bad[:8]}")
        for k in bad[:8]:
            d = (a[k].double() - b[k].double()).abs()
            print(f"  {k}: max |diff| {float(d.nan_to_num(1e9).max()):.3e}, "
                  f"{int((d > 0).sum())} elements")
        sys.exit(1 if bad else 0)
