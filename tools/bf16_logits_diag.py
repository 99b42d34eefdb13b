"""Diagnosis (tool, CPU only): where does the bf16 C2 step lose 2-5% of gradient direction
against the fp32 oracle (test_c2_training_step_bf16_vs_oracle)?

The oracle's fp32 forward (tests/test_gpu_parity_step.py's conditioned init, B=2, T=1500, seed 6
as the test) gives logits; the CTC gradient is taken (fp64) on the logits as they are and on a
perturbed copy, and each is pushed through the SAME fp32 encoder backward.  Cosine / norm ratio
per tensor between the two = the loss that perturbation of the logits alone causes, with every
other part of the step exact.  Perturbations:
  round   the logits rounded to bf16 (what a bf16 output projection stores)
  operand fp32 logits from bf16-rounded operands (hidden and Wo rounded, fp32 accumulation: what
          an fp32-output GEMM under bf16 autocast computes)
  noise   fp32 logits + N(0, (2^-9 |logit|)^2) noise (rounding-sized, unbiased)
  +exact  round / operand with the emission columns (blank and the sequence's labels) exact
All three give the same 2-5% loss: at this init the CTC gradient over T=1500 frames is that
sensitive to any perturbation of bf16 size in the logits (MEASURED on MI355X too: an fp32-output
projection, ops.CTCHeadFn, moved the cosines by < 0.01 either way, profiles/r4_parity_measured.md).

    python tools/bf16_logits_diag.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import ctc as octc, lucy_step  # noqa: E402
from tests.test_gpu_parity_step import D512, L6, oracle_params, step_inputs  # noqa: E402


def grads_for(p, logits, tok, in_lens, U, x, caches, h, s):
    nll, grad = octc.ctc_loss_grad(logits, tok, in_lens, U, blank=0, logits=True)
    scale = octc.ctc_mean_grad_scale(nll, U)
    dlog = (grad * scale[:, None, None]).astype(np.float32)
    return lucy_step.encoder_backward(p, dlog, x, caches, h, s, L6, D512)


def main():
    B, T = 2, 1500
    p = oracle_params()
    feats, tok, U = step_inputs(B, T, 6)
    in_lens = np.full(B, T)
    logits, _, x, (caches, h, s) = lucy_step.forward(p, feats, L6, D512)
    ref = grads_for(p, logits, tok, in_lens, U, x, caches, h, s)
    lb = lucy_step._bf16(logits).astype(np.float32)
    print(f"logits: std {logits.std():.3f}, |bf16 - fp32| max {np.abs(lb - logits).max():.2e}")
    bf = lambda a: lucy_step._bf16(a).astype(np.float32)   # noqa: E731
    lo = (bf(x.reshape(-1, D512)) @ bf(p["Wo"]).T + p["bo"]).reshape(logits.shape).astype(np.float32)
    rng = np.random.default_rng(0)
    ln = (logits * (1 + 2.0 ** -9 * rng.standard_normal(logits.shape))).astype(np.float32)
    # the same with the emission columns (blank + the sequence's labels) exact: what a bf16
    # output projection plus exact emission logits would feed the loss
    emis = np.zeros((B, 1, logits.shape[-1]), bool)
    for b in range(B):
        emis[b, 0, 0] = True
        emis[b, 0, np.asarray(tok[b][:U[b]])] = True
    lbx = np.where(emis, logits, lb).astype(np.float32)
    lox = np.where(emis, logits, lo).astype(np.float32)
    names = ("round", "operand", "noise", "round+exact", "operand+exact")
    res = {}
    for name, lg in zip(names, (lb, lo, ln, lbx, lox)):
        print(f"{name}: |logits - fp32| rms {np.sqrt(((lg - logits) ** 2).mean()):.2e}")
        got = grads_for(p, lg, tok, in_lens, U, x, caches, h, s)
        for k in ref:
            g, r = got[k].ravel().astype(np.float64), ref[k].ravel().astype(np.float64)
            res.setdefault(k, []).append((g @ r / (np.linalg.norm(g) * np.linalg.norm(r)),
                                          np.linalg.norm(g) / np.linalg.norm(r)))
    print("tensor   " + "   ".join(f"{n:>13s} cos / ratio" for n in names))
    for k, v in res.items():
        print(f"{k:4s}     " + "   ".join(f"      {c:.4f} / {q:.4f}" for c, q in v))


if __name__ == "__main__":
    main()
