"""clip_grad_norm_ + Adam / AdamW step on HIP (csrc/optim.hip) for the segment loop's optimizer
step (/root/reference/train.py:543-552; the optimizers of train.py:112-136).

``clip_and_adam_step(optimizer, clip_params, max_norm)`` does what

    torch.nn.utils.clip_grad_norm_(clip_params, max_norm)
    optimizer.step()

does for a ``torch.optim.Adam`` / ``AdamW`` built the way the reference builds them (default
``foreach`` / single-tensor implementation), in two launches:

* ``sc_adam_sumsq``: per-chunk sums of squares of the clipped gradients (fixed order);
* ``sc_adam_step``: the clip coefficient (every workgroup reduces the chunk sums the same way),
  then one pass over p, g, exp_avg, exp_avg_sq per parameter group.

The optimizer's state is torch's own (``state[p]["step"]`` a CPU float32 tensor,
``exp_avg``, ``exp_avg_sq``), so ``optimizer.state_dict()`` / ``load_state_dict`` and LR
schedulers (they write ``group["lr"]``) work unchanged, and either implementation may take the
next step.  Parameters outside ``clip_params`` (e.g. an RNN-T joiner in the same optimizer:
the reference clips ``model.parameters()`` only) are stepped unclipped.  ``p.grad`` is read
only: it keeps its unclipped values (the loop zeroes it right after).

``hip_adam_eligible(optimizer)`` says whether this path applies; otherwise the caller uses
torch's clip + step.  Never a silent fallback inside: a call on an ineligible optimizer raises.
"""
import math

import torch
from torch.autograd.graph import increment_version

from . import _lib
from ._lib import AdamTensor, check, ptr, stream_of


def _group_ok(g):
    return (not g.get("amsgrad", False) and not g.get("maximize", False)
            and not g.get("capturable", False) and not g.get("differentiable", False)
            and not g.get("fused", False) and not isinstance(g["lr"], torch.Tensor)
            and not isinstance(g["betas"][0], torch.Tensor)
            and not isinstance(g["betas"][1], torch.Tensor))


def _param_ok(p, state):
    if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
        return False
    g = p.grad
    if g is not None and (g.is_sparse or g.dtype != torch.float32 or g.device != p.device):
        return False
    if state:
        st = state.get("step")
        m, v = state.get("exp_avg"), state.get("exp_avg_sq")
        if (st is None or (isinstance(st, torch.Tensor) and st.device.type != "cpu")
                or m is None or v is None or "max_exp_avg_sq" in state
                or not (m.is_contiguous() and v.is_contiguous())
                or m.dtype != torch.float32 or v.dtype != torch.float32):
            return False
    return True


def hip_adam_eligible(optimizer) -> bool:
    """True for a torch.optim.Adam / AdamW (not fused, capturable, amsgrad, maximize or
    differentiable; scalar lr and betas) over fp32 contiguous ROCm parameters whose state, if
    any, is torch's non-fused layout."""
    if type(optimizer) not in (torch.optim.Adam, torch.optim.AdamW):
        return False
    for g in optimizer.param_groups:
        if not _group_ok(g):
            return False
        for p in g["params"]:
            if not _param_ok(p, optimizer.state.get(p)):
                return False
    return True


def _entry(p, state):
    if not state:   # torch's lazy state init (Adam._init_group, non-fused, non-capturable)
        state["step"] = torch.tensor(0.0, dtype=torch.float32)
        state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
    g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
    return AdamTensor(p.data_ptr(), g.data_ptr(), state["exp_avg"].data_ptr(),
                      state["exp_avg_sq"].data_ptr(), p.numel()), g


def _table(entries):
    return (AdamTensor * max(1, len(entries)))(*entries)


@torch.no_grad()
def clip_and_adam_step(optimizer, clip_params, max_norm):
    """clip_grad_norm_(clip_params, max_norm) + optimizer.step() on HIP.  Returns the total
    gradient norm of clip_params (0-dim fp32 device tensor), as clip_grad_norm_ does."""
    if not hip_adam_eligible(optimizer):
        raise RuntimeError("clip_and_adam_step: optimizer not supported by the HIP Adam path "
                           "(hip_adam_eligible is False)")
    lib = _lib.load()
    default_decoupled = type(optimizer) is torch.optim.AdamW
    clip_ids = {id(p) for p in clip_params}
    groups, keep = [], []
    clip_entries = []
    dev = None
    for g in optimizer.param_groups:
        members = []
        for p in g["params"]:
            if p.grad is None:
                continue
            e, gc = _entry(p, optimizer.state[p])
            keep.append(gc)
            members.append((p, e))
            if id(p) in clip_ids:
                clip_entries.append(e)
            dev = p.device
        groups.append((g, members))
    if dev is None:
        return torch.zeros((), dtype=torch.float32)
    stream = stream_of(keep[0])
    part, nparts = None, 0
    if clip_entries:
        tab = _table(clip_entries)
        nparts = lib.sc_adam_parts(tab, len(clip_entries))
        if nparts:
            part = torch.empty(nparts, dtype=torch.float32, device=dev)
            check(lib.sc_adam_sumsq(tab, len(clip_entries), ptr(part), stream), "sc_adam_sumsq")
    # the first clipped sc_adam_step launch writes the norm; with nothing to clip it is 0
    norm = torch.empty(1, dtype=torch.float32, device=dev) if part is not None else \
        torch.zeros(1, dtype=torch.float32, device=dev)
    norm_out = norm
    for g, members in groups:
        beta1, beta2 = g["betas"]
        wd = g.get("weight_decay", 0.0)
        lr = g["lr"]
        # torch.optim.Adam(..., decoupled_weight_decay=True) is AdamW's update (torch >= 2.6
        # stores the flag per group; AdamW sets it too): p *= 1 - lr wd instead of g += wd p
        decoupled = 1 if g.get("decoupled_weight_decay", default_decoupled) else 0
        # parameters of one group share a step count unless added mid-training: one launch per
        # (clipped?, step) class
        classes = {}
        for p, e in members:
            st = optimizer.state[p]["step"]
            st += 1
            step = float(st)
            classes.setdefault((id(p) in clip_ids, step), []).append(e)
        for (clipped, step), ents in classes.items():
            bc1 = 1.0 - beta1 ** step
            bc2 = 1.0 - beta2 ** step
            use_part = part if (clipped and part is not None) else None
            rc = lib.sc_adam_step(_table(ents), len(ents), ptr(use_part), nparts if use_part is not None else 0,
                                  float(max_norm), float(lr), float(beta1), float(beta2),
                                  float(g["eps"]), float(wd), decoupled, lr / bc1, math.sqrt(bc2),
                                  ptr(norm_out) if use_part is not None else None, stream)
            check(rc, "sc_adam_step")
            if use_part is not None:
                norm_out = None
        increment_version([p for p, _ in members])   # parameters changed in place
    return norm[0]
