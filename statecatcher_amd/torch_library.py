"""The hot-path ops as dispatcher ops: ``torch.ops.statecatcher.*`` (csrc/torch_ops.cpp,
``TORCH_LIBRARY(statecatcher, m)``).

The C++ extension registers each op's schema, its HIP kernel (CUDA dispatch key) and a Meta
kernel (shapes only).  This module loads it and registers the autograd formulas over the
``*_bwd`` ops, so the functions below are differentiable, traceable by FakeTensor /
``torch.compile(fullgraph=True)`` and checkable with ``torch.library.opcheck``.  They launch the
same kernels as the ctypes autograd nodes of ``ops.py`` (the training hot path), which stay the
lower-overhead route for eager training.

Reference interfaces (what a ``train.py`` user swaps in):
  lucy_scan   <- rnn_forward_unfused_rmsnorm                        lucyrnn_triton.py:61-73, :180-244
  decay_scan  <- fused_decay_scan                                    lucyrnn_triton.py:158-177
  layer_norm  <- nn.LayerNorm(D) between layers                      lucyrnn_triton.py:96-97, :136-137
  ctc_loss    <- nn.CTCLoss(blank, reduction='mean', zero_infinity)  train.py:142 (on model.py:70's
                 log_softmax, fused here when is_logits)
  ctc_greedy_decode <- decoder.py:3-30
  mlstm       <- the xLSTM encoder's mLSTM cell (fork mlstm_kernels)  model.py:214-229
  rnnt_joint_nll <- RNNTPredictorJoiner + log_softmax + warp_rnnt      model.py:73-145
  gemm_tn     <- LinearSafe's forward / input-gradient GEMM (bf16)    lucyrnn_triton.py:20-25
  gemm_wgrad  <- LinearSafe / output_proj weight gradient             lucyrnn_triton.py:20-25, :107-109
  clip_adam_  <- clip_grad_norm_(params, 50) + optim.Adam/AdamW.step() train.py:543-552
"""
import os

import torch

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_torch_ops.so")
OPS = ("abi_version", "lucy_scan_fwd", "lucy_scan_bwd", "decay_scan_fwd", "decay_scan_bwd",
       "layer_norm_fwd", "layer_norm_bwd", "ctc_fwd", "ctc_bwd", "ctc_mean", "ctc_greedy_decode",
       "mlstm_fwd", "mlstm_bwd", "mlstm_gate_bwd", "rnnt_joint_fwd", "rnnt_joint_bwd",
       "gemm_tn", "gemm_wgrad", "clip_adam_")

_LOADED = False


def load():
    """Load the extension (once) and register the autograd formulas.  Raises if it is not built:
    there is no Python fallback for these ops."""
    global _LOADED
    if _LOADED:
        return torch.ops.statecatcher
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"statecatcher TORCH_LIBRARY extension not built: {LIB_PATH} missing "
                           "(make -C statecatcher_amd/csrc)")
    torch.ops.load_library(LIB_PATH)
    _register_autograd()
    _LOADED = True
    return torch.ops.statecatcher


# ------------------------------------------------------------------------------- autograd -----
def _scan_setup(ctx, inputs, output):
    gates, h0, s0, bias, need_ckpt = inputs
    ctx.save_for_backward(gates, output[3], bias)
    ctx.has_bias = bias is not None
    ctx.dtypes = (h0.dtype, s0.dtype, None if bias is None else bias.dtype)


def _scan_backward(ctx, dout, ds_last, dh_last, dckpt):
    gates, ckpt, bias = ctx.saved_tensors
    sc = torch.ops.statecatcher
    B, T = gates.shape[:2]
    D = gates.shape[-1] if gates.dim() == 4 else gates.shape[2] * 64
    if dout is None:
        dout = gates.new_zeros(B, T, D)
    if dh_last is not None:   # h_last is out[:, -1] before rounding: its gradient joins dout's
        dout = dout.clone()
        dout[:, -1] += dh_last.to(dout.dtype)
    want_db = ctx.has_bias and ctx.needs_input_grad[3]
    dgates, dh0, ds0, dbias = sc.lucy_scan_bwd(gates, ckpt, dout, ds_last, bias, want_db)
    hd, sd, bd = ctx.dtypes
    db = None
    if want_db:   # per-row partials [B,7,D] -> the bias's [7,D] (logical g*D + d) order
        db = dbias.sum(0).reshape(bias.shape).to(bd)
    return dgates, dh0.to(hd), ds0.to(sd), db, None


def _decay_setup(ctx, inputs, output):
    kv, decay, init = inputs
    ctx.save_for_backward(decay, output, init)
    ctx.init_dtype = None if init is None else init.dtype


def _decay_backward(ctx, dout):
    decay, s_all, init = ctx.saved_tensors
    dkv, ddec, dinit = torch.ops.statecatcher.decay_scan_bwd(decay, s_all, dout, init)
    return dkv, ddec.to(decay.dtype), (dinit.to(ctx.init_dtype) if init is not None else None)


def _ln_setup(ctx, inputs, output):
    x, gamma, beta, eps = inputs
    ctx.save_for_backward(x, gamma, output[1], output[2])
    ctx.pdtypes = (gamma.dtype, beta.dtype)


def _ln_backward(ctx, dy, dmean, drstd):
    x, gamma, mean, rstd = ctx.saved_tensors
    dx, dg, db = torch.ops.statecatcher.layer_norm_bwd(x, dy, gamma, mean, rstd)
    gd, bd = ctx.pdtypes
    return dx, dg.to(gd), db.to(bd), None


def _ctc_setup(ctx, inputs, output):
    x, targets, in_lens, tgt_lens, blank, is_logits = inputs
    ctx.save_for_backward(x, targets, in_lens, tgt_lens, output[0], output[1])
    ctx.meta = (blank, is_logits)


def _ctc_backward(ctx, grad_nll, grad_ws):
    x, targets, in_lens, tgt_lens, nll, ws = ctx.saved_tensors
    blank, is_logits = ctx.meta
    if grad_nll is None:
        return None, None, None, None, None, None
    grad = torch.ops.statecatcher.ctc_bwd(x, targets, in_lens, tgt_lens, nll, ws, grad_nll,
                                          blank, is_logits)
    return grad, None, None, None, None, None


def _mean_setup(ctx, inputs, output):
    ctx.save_for_backward(output[1])


def _mean_backward(ctx, grad_loss, grad_factor):
    (factor,) = ctx.saved_tensors
    return (factor * grad_loss if grad_loss is not None else None), None


def _mlstm_setup(ctx, inputs, output):
    q, k, v, ig, fg, c0, n0, m0, eps = inputs
    h, c_last, ns, ms, cs, mrow, den = output
    ctx.save_for_backward(q, k, v, ig, fg, h, cs, ns, ms, mrow, den)
    ctx.eps = eps
    ctx.has = (c0 is not None, n0 is not None)
    ctx.nc = ns.shape[1] - 1


def _mlstm_backward(ctx, dh, dc_last, dns, dms, dcs, dmrow, dden):
    """Gradients of (h, final C, final n) -- the n / m state outputs beyond the final chunk are
    internal (their gradients are ignored, as the stabiliser is not differentiated)."""
    q, k, v, ig, fg, h, cs, ns, ms, mrow, den = ctx.saved_tensors
    if dh is None:
        dh = torch.zeros_like(h)
    dn_last = None if dns is None else dns[:, ctx.nc].reshape(q.shape[0], q.shape[1], -1)
    dq, dk, dv, dc0, dn0, qdq, kdk = torch.ops.statecatcher.mlstm_bwd(
        q, k, v, ig, fg, h, dh, dc_last, dn_last, cs, ns, ms, mrow, den, ctx.eps)
    # d igate_s = k_s.dk_s ; d fgate_t = sigmoid(-f_t) sum_{r >= t} (q_r.dq_r - k_r.dk_r)
    dfg = torch.ops.statecatcher.mlstm_gate_bwd(qdq, kdk, fg)
    has_c0, has_n0 = ctx.has
    return (dq, dk, dv, kdk.to(ig.dtype), dfg.to(fg.dtype), dc0 if has_c0 else None,
            dn0 if has_n0 else None, None, None)


def _joint_setup(ctx, inputs, output):
    enc, pred, W, bias, labels, flen, llen, blank = inputs
    ctx.save_for_backward(enc, pred, W, bias, labels, flen, llen, output[1])
    ctx.blank = blank
    ctx.dtypes = (enc.dtype, pred.dtype, W.dtype, bias.dtype)


def _joint_backward(ctx, grad_nll, grad_ws):
    enc, pred, W, bias, labels, flen, llen, ws = ctx.saved_tensors
    if grad_nll is None:
        return (None,) * 8
    de, dp, dW, db = torch.ops.statecatcher.rnnt_joint_bwd(enc, pred, W, bias, labels, flen, llen,
                                                           ws, grad_nll, ctx.blank)
    ed, pd, wd, bd = ctx.dtypes
    return de.to(ed), dp.to(pd), dW.to(wd), db.to(bd), None, None, None, None


def _register_autograd():
    reg = torch.library.register_autograd
    reg("statecatcher::lucy_scan_fwd", _scan_backward, setup_context=_scan_setup)
    reg("statecatcher::decay_scan_fwd", _decay_backward, setup_context=_decay_setup)
    reg("statecatcher::layer_norm_fwd", _ln_backward, setup_context=_ln_setup)
    reg("statecatcher::ctc_fwd", _ctc_backward, setup_context=_ctc_setup)
    reg("statecatcher::ctc_mean", _mean_backward, setup_context=_mean_setup)
    reg("statecatcher::mlstm_fwd", _mlstm_backward, setup_context=_mlstm_setup)
    reg("statecatcher::rnnt_joint_fwd", _joint_backward, setup_context=_joint_setup)


# ------------------------------------------------------------------------------- functions ----
def lucy_scan(gates, h0, s0, gate_bias=None):
    """(out [B,T,D] in gates' dtype, s_last fp32, h_last fp32) of the LucyRNN scan over gates
    [B,T,7,D] (the reference layout) or step-blocked [B,T,D/64,7,64]; gate_bias fp32 [7,D] is
    added on load.  Differentiable in gates, h0, s0 and gate_bias."""
    sc = load()
    need = torch.is_grad_enabled() and any(
        t is not None and t.requires_grad for t in (gates, h0, s0, gate_bias))
    out, s_last, h_last, _ = sc.lucy_scan_fwd(gates, h0, s0, gate_bias, need)
    return out, s_last, h_last


def decay_scan(kv, decay, init=None):
    """s_t = decay_t s_{t-1} + kv_t with s_{-1} = init (zeros if None); fused_decay_scan."""
    return load().decay_scan_fwd(kv, decay, init)


def layer_norm(x, gamma, beta, eps=1e-5):
    """nn.LayerNorm over the last dim in x's dtype with fp32 statistics."""
    return load().layer_norm_fwd(x, gamma, beta, eps)[0]


def ctc_nll(x, targets, in_lens, tgt_lens, blank=0, is_logits=True):
    """Per-sequence CTC negative log-likelihood [B] fp32 (+inf when infeasible)."""
    return load().ctc_fwd(x, targets, in_lens, tgt_lens, blank, is_logits)[0]


def ctc_loss(x, targets, in_lens, tgt_lens, blank=0, is_logits=True):
    """nn.CTCLoss(blank, reduction='mean', zero_infinity=True) (train.py:142)."""
    sc = load()
    nll = sc.ctc_fwd(x, targets, in_lens, tgt_lens, blank, is_logits)[0]
    return sc.ctc_mean(nll, tgt_lens)[0]


def ctc_greedy_decode(log_probs, lengths, blank=0):
    """(tokens int32 [B,T], counts int32 [B]) of decoder.py's greedy CTC decode."""
    return load().ctc_greedy_decode(log_probs, lengths, blank)


def mlstm(q, k, v, igate, fgate, c0=None, n0=None, m0=None, eps=1e-6):
    """transformers' mlstm_chunkwise(return_last_states=True) on the HIP walk kernels:
    (h [B,NH,T,DV], (C [B,NH,DQ,DV], n [B,NH,DQ], m [B,NH,1])).  q, k, v bf16 / f16, gates fp32
    [B,NH,T]; differentiable in q, k, v, the gates, c0 and n0."""
    h, c_last, ns, ms, _, _, _ = load().mlstm_fwd(q, k, v, igate, fgate, c0, n0, m0, eps)
    B, NH = q.shape[:2]
    return h, (c_last, ns[:, -1].reshape(B, NH, -1), ms[:, -1].reshape(B, NH, 1))


def rnnt_joint_nll(enc_p, pred_p, W, bias, labels, frames_lengths, labels_lengths, blank=0):
    """Per-sequence RNN-T nll [B] of the fused joiner (RNNTPredictorJoiner's joint, log_softmax,
    warp_rnnt's gathered lattice) without materialising the (B, T, U+1, V) logits."""
    return load().rnnt_joint_fwd(enc_p, pred_p, W, bias, labels, frames_lengths, labels_lengths,
                                 blank)[0]


def gemm_tn(a, b, tile_m=0):
    """C [M,N] bf16 = a [M,K] b [N,K]^T on the persistent MFMA kernel (K % 64 == 0, N % 256 == 0;
    include/statecatcher.h sc_gemm_tn_bf16).  Not differentiable: a building block of the
    projection nodes' forward and input gradient."""
    return load().gemm_tn(a, b, tile_m)


def gemm_wgrad(dy, x, block_d=0):
    """dW [N,K] fp32 = dy [M,N]^T x [M,K] (bf16 operands) on the split-L MFMA kernel plus the
    fixed-order slab sum; block_d = D: dy's columns in step-blocked gate order, dW returned in
    the reference's row order.  Raises outside the kernel's tiling (sc_gemm_wgrad_splits)."""
    return load().gemm_wgrad(dy, x, block_d)


def clip_adam_(params, grads, exp_avgs, exp_avg_sqs, n_clip, max_norm, lr, betas, eps,
               weight_decay, decoupled, step):
    """clip_grad_norm_(params[:n_clip], max_norm) then one Adam (decoupled=False) / AdamW step
    at step count `step` on every tensor, in place (params, exp_avgs, exp_avg_sqs; grads read
    only), as optim.clip_and_adam_step does for an optimizer.  Returns clip_grad_norm_'s total
    norm (0-dim fp32 tensor; 0 without clipping)."""
    import math
    beta1, beta2 = betas
    bc1, bc2 = 1.0 - beta1 ** step, 1.0 - beta2 ** step
    return load().clip_adam_(list(params), list(grads), list(exp_avgs), list(exp_avg_sqs),
                             int(n_clip), float(max_norm), float(lr), float(beta1), float(beta2),
                             float(eps), float(weight_decay), bool(decoupled), lr / bc1,
                             math.sqrt(bc2))
