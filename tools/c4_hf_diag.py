#!/usr/bin/env python3
"""Diagnostic: the full 12-block C4 encoder (default init, B = 1, T = 1536) against transformers'
xLSTMBlock composition in fp64 on the GPU, per block: relative Frobenius error of the q / k /
out_proj weight gradients for ours (bf16 cell, core path), ours (bf16 cell, split path), ours
(fp16 cell) and transformers' own bf16-autocast run.  Cotangent: a fixed random R on the
soft-capped logits (tests/test_gpu_c4._slice_ref).
usage: python tools/c4_hf_diag.py [--t 1536]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import test_gpu_c4 as c4   # noqa: E402
from statecatcher_amd import ops   # noqa: E402

DEV = c4.DEV = torch.device("cuda:0")
T = int(sys.argv[sys.argv.index("--t") + 1]) if "--t" in sys.argv else 1536
NB = 12
NAMES = ["mlstm_layer.q.weight", "mlstm_layer.k.weight", "mlstm_layer.out_proj.weight",
         "ffn.proj_down.weight"]


def hf_grads(state, x, R, autocast):
    from transformers import xLSTMConfig
    from transformers.models.xlstm import modeling_xlstm as M
    cfg = xLSTMConfig(hidden_size=768, embedding_dim=768, num_heads=4, num_blocks=NB,
                      vocab_size=c4.V, mode="train", chunkwise_kernel="chunkwise--native_autograd",
                      autocast_kernel_dtype="float32", return_last_states=True)
    dt = torch.float32 if autocast else torch.float64
    hf = torch.nn.ModuleList([M.xLSTMBlock(cfg) for _ in range(NB)])
    hf.load_state_dict({k[len("encoder.blocks."):]: v for k, v in state.items()
                        if k.startswith("encoder.blocks.")})
    hf = hf.to(DEV, dt)
    norm = M.xLSTMRMSNorm(768, eps=cfg.norm_eps)
    norm.load_state_dict({"weight": state["encoder.out_norm.weight"]})
    norm = norm.to(DEV, dt)
    W_e = state["encoder.embedding.weight"].to(DEV, dt)
    b_e = state["encoder.embedding.bias"].to(DEV, dt)
    W_l = state["encoder.lm_head.weight"].to(DEV, dt)
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        h = torch.nn.functional.linear(x.to(DEV, dt), W_e, b_e)
        for blk in hf:
            h, _ = blk(h)
        ref = torch.nn.functional.linear(norm(h), W_l)
    ref = 30.0 * torch.tanh(ref.to(dt) / 30.0)
    (ref * R.to(DEV, dt)).sum().backward()
    return {f"{i}.{n}": dict(hf[i].named_parameters())[n].grad.double() for i in range(NB)
            for n in NAMES}


def ours(state, x, R, kdt, split):
    model = c4.c4_model(kdt, blocks=NB, seed=0)
    model.load_state_dict(state)
    orig = ops.mlstm_core_supported
    if split:
        ops.mlstm_core_supported = lambda *a: False
    try:
        xd = x.to(DEV)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits, _ = model(xd, None)
        (logits.float() * R.to(DEV)).sum().backward()
    finally:
        ops.mlstm_core_supported = orig
    blocks = model.encoder.blocks
    return {f"{i}.{n}": dict(blocks[i].named_parameters())[n].grad.double() for i in range(NB)
            for n in NAMES}


state = {k: v.detach().cpu() for k, v in c4.c4_model("bfloat16", blocks=NB, seed=0).state_dict().items()}
g = torch.Generator().manual_seed(9)
x = torch.randn(1, T, c4.F, generator=g)
R = torch.randn(1, T, c4.V, generator=g)
exact = hf_grads(state, x, R, False)
runs = {"hf-bf16": hf_grads(state, x, R, True),
        "ours-bf16-core": ours(state, x, R, "bfloat16", False),
        "ours-bf16-split": ours(state, x, R, "bfloat16", True),
        "ours-fp16": ours(state, x, R, "float16", True)}
for key in exact:
    e = exact[key]
    line = " | ".join(f"{name} {float((r[key] - e).norm() / e.norm()):.2e}" for name, r in runs.items())
    print(f"block {key}: |g| {float(e.norm()):.3e} | {line}", flush=True)
