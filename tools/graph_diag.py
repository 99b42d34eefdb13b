"""Diagnostic (GPU): where do graph-replayed segments first differ from the eager ones?
Per segment position, the gradients of forward_backward (no optimizer step in between), then the
parameters after one clip + Adam step.  Usage: python tools/graph_diag.py [ctc|rnnt]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_gpu_graphs import _segments, _trainer  # noqa: E402
from statecatcher_amd.graphs import GraphedSegments  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "rnnt"
cfg = dict(ctc=(3, 256, 256, 4, 300, 20), rnnt=(2, 256, 256, 2, 200, 12))[mode]
L, H, V, B, T, U = cfg
segs = _segments(3, B, T, V, U, seed=9)


def named(tr):
    names = {id(p): n for n, p in tr.model.named_parameters()}
    if tr.joiner is not None:
        names.update({id(p): "joiner." + n for n, p in tr.joiner.named_parameters()})
    return names


def report(tag, a, b, names, params):
    bad = 0
    for p, x, y in zip(params, a, b):
        if x is None or y is None:
            if (x is None) != (y is None):
                print(f"  {tag} {names[id(p)]}: None mismatch")
            continue
        if not torch.equal(x, y):
            bad += 1
            d = (x.double() - y.double()).abs()
            print(f"  {tag} {names[id(p)]}: max |diff| {float(d.max()):.3e} "
                  f"({int((d > 0).sum())} of {d.numel()} elements), |x| max {float(x.abs().max()):.3e}")
    print(f"{tag}: {bad} tensors differ")


tr_e, p_e = _trainer(mode, L, H, V)
tr_g, p_g = _trainer(mode, L, H, V)
names = named(tr_g)
gs = GraphedSegments(tr_g, segs).capture()
params = gs.params

# eager twice: is the eager path itself deterministic?
ge = []
for rep in range(2):
    st = None
    out = []
    for i in range(3):
        for p in tr_e.optimizer.param_groups[0]["params"]:
            p.grad = None
        s = segs[i]
        loss, st = tr_e.forward_backward(s["feats"], s["masks"], s["tokens"], s["in_lens"],
                                         s["tgt_lens"], st)
        out.append(([p.grad.clone() if p.grad is not None else None for p in
                     [q for g in tr_e.optimizer.param_groups for q in g["params"]]], loss.clone()))
    ge.append(out)
torch.cuda.synchronize()
for i in range(3):
    report(f"eager-vs-eager seg{i}", ge[0][i][0], ge[1][i][0], names, params)
for i in range(3):
    gs.graphs[i].replay()
    torch.cuda.synchronize()
    print(f"seg{i} loss eager {float(ge[0][i][1].detach()):.6f} graph {float(gs.losses[i].detach()):.6f}")
    report(f"eager-vs-graph seg{i}", ge[0][i][0], gs.grads[i], names, params)

# with optimizer steps: fresh trainers, segment 0 + step, then segment 1's gradients
tr_e, _ = _trainer(mode, L, H, V)
tr_g, _ = _trainer(mode, L, H, V)
gs = GraphedSegments(tr_g, segs).capture()
pe = [q for g in tr_e.optimizer.param_groups for q in g["params"]]
tr_e.begin_batch()
s = segs[0]
tr_e.train_segment(s["feats"], s["masks"], s["tokens"], s["in_lens"], s["tgt_lens"])
gs.begin_batch()
gs.step()
torch.cuda.synchronize()
report("after step 1: params", [p.detach() for p in pe], [p.detach() for p in gs.params], names,
       gs.params)
st = [ (t.detach() if torch.is_tensor(t) else t) for t in []]
s = segs[1]
for p in pe:
    p.grad = None
loss_e, _ = tr_e.forward_backward(s["feats"], s["masks"], s["tokens"], s["in_lens"], s["tgt_lens"],
                                  tr_e.encoder_state)
gs.graphs[1].replay()
torch.cuda.synchronize()
print(f"seg1 after one step: loss eager {float(loss_e.detach()):.6f} graph {float(gs.losses[1].detach()):.6f}")
report("seg1 grads after step 1", [p.grad for p in pe], gs.grads[1], names, gs.params)
