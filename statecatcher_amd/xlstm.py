"""xLSTM encoder (config C4) around the HIP mLSTM cell (csrc/mlstm.hip).

The reference builds ``xLSTMLarge(xLSTMLargeConfig(...))`` from its fork of NX-AI's xlstm
package (model.py:214-229, :301-307; the fork adds ``input_dim``).  The fork is not available
(parity w.r.t. the fork unpinned); the block structure here is the published
xLSTM-large architecture as transformers 5.15.0 restates it
(transformers/models/xlstm/modeling_xlstm.py:870-1205), with the same parameter names:

  block:  x + mLSTMLayer(RMSNorm(x));  x + FFN(RMSNorm(x))
  layer:  q, k, v, o = Linear(x);  i, f = softcap(Linear(x), 15)  (one gate per head)
          h = mLSTM cell (HIP, chunkwise, state carried);  y = out_proj(sigmoid(o) *
          MultiHeadLayerNorm(h))
  FFN:    proj_down(silu(proj_up_gate(x)) * proj_up(x))
  model:  input projection (the fork's input_dim -> embedding_dim; a Linear named
          ``embedding``), blocks, out_norm, lm_head, logits softcap(30)

Recurrent state: {block index: (C [B,NH,DQ,DV], n [B,NH,DQ], m [B,NH,1])}, carried across
segments like LucyRNNtriton's (detach_states handles dicts).  Sequences must be a multiple of
the 64-step chunk: ASRModel pads to 64 exactly as the reference does (model.py:341-347).
"""
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .ops import mlstm_chunkwise


def _linear(x, w, b=None, bias_from=0):
    """nn.Linear under autocast; on the GPU through ops.autocast_linear, whose backward takes the
    weight gradient (a reduction over all B*T rows) from the MFMA split-L kernel.  bias_from:
    b[:bias_from] are constant zero pieces whose gradient is not summed."""
    if x.is_cuda:
        return ops.autocast_linear(x, w, b, bias_from)
    return F.linear(x, w, b)


_ZEROS = {}


def _zeros(n, dtype, device):
    """A cached zero bias piece (read only): the concatenated projection bias of the bias-free
    q / k / v / o Linears takes no fill launch per call."""
    key = (n, dtype, str(device))
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros(n, dtype=dtype, device=device)
    return z


def soft_cap(x, cap):
    return x if cap is None else cap * torch.tanh(x / cap)


def round_up(x, m):
    return int(((x + m - 1) // m) * m)


@dataclass
class xLSTMLargeConfig:
    """Fields the reference passes (model.py:216-228) plus xLSTM-large's defaults."""
    embedding_dim: int
    num_heads: int
    num_blocks: int
    vocab_size: int
    input_dim: Optional[int] = None
    return_last_states: bool = True
    mode: str = "train"
    chunkwise_kernel: str = "chunkwise--native_autograd"
    sequence_kernel: str = "native_sequence__native"
    step_kernel: str = "native"
    autocast_kernel_dtype: str = "bfloat16"
    qk_dim_factor: float = 0.5
    v_dim_factor: float = 1.0
    gate_soft_cap: float = 15.0
    output_logit_soft_cap: float = 30.0
    norm_eps: float = 1e-6
    norm_reduction_force_float32: bool = True
    ffn_proj_factor: float = 2.667
    ffn_round_up_to_multiple_of: int = 64
    use_bias: bool = False
    add_out_norm: bool = True
    eps: float = 1e-6
    chunk_size: int = 64


class RMSNorm(nn.Module):
    def __init__(self, num_features, eps=1e-6, use_bias=False, force_float32_reductions=True):
        super().__init__()
        self.eps = eps
        self.force_float32_reductions = force_float32_reductions
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features)) if use_bias else None

    def forward(self, x):
        if (self.bias is None and self.force_float32_reductions
                and ops.xlstm_glue_supported(x, x.shape[-1])):
            # one HIP pass (csrc/xlstm_glue.hip), same roundings; bf16 out = what autocast would
            # hand the next GEMM
            return ops.rms_norm(x, self.weight, self.eps)
        dt = x.dtype
        y = x.float() if self.force_float32_reductions else x
        y = (y * torch.rsqrt(y.pow(2).mean(-1, keepdim=True) + self.eps)).to(dt)
        y = y * self.weight
        return y + self.bias if self.bias is not None else y


class MultiHeadLayerNorm(nn.Module):
    def __init__(self, num_heads, head_dim, eps=1e-6, use_bias=False, force_float32_reductions=True):
        super().__init__()
        self.num_heads, self.head_dim, self.eps = num_heads, head_dim, eps
        self.force_float32_reductions = force_float32_reductions
        self.weight = nn.Parameter(torch.ones(num_heads * head_dim))
        self.bias = nn.Parameter(torch.zeros(num_heads * head_dim)) if use_bias else None

    def forward(self, x):   # x [B, T, NH, DH]
        B, T = x.shape[:2]
        dt = x.dtype
        y = x.float() if self.force_float32_reductions else x
        y = (y - y.mean(-1, keepdim=True)) * torch.rsqrt(y.var(-1, keepdim=True, unbiased=False) + self.eps)
        y = y.to(dt).reshape(B, T, -1) * self.weight
        return y + self.bias if self.bias is not None else y


class FeedForward(nn.Module):
    def __init__(self, cfg: xLSTMLargeConfig):
        super().__init__()
        up = round_up(cfg.embedding_dim * cfg.ffn_proj_factor, cfg.ffn_round_up_to_multiple_of)
        self.proj_up_gate = nn.Linear(cfg.embedding_dim, up, bias=cfg.use_bias)
        self.proj_up = nn.Linear(cfg.embedding_dim, up, bias=cfg.use_bias)
        self.proj_down = nn.Linear(up, cfg.embedding_dim, bias=cfg.use_bias)

    def forward(self, x):
        # proj_up_gate and proj_up as ONE GEMM over the concatenated weight (parameters and
        # state_dict unchanged): one read and one autocast cast of x instead of two
        up = self.proj_up.weight.shape[0]
        ws = [self.proj_up_gate.weight, self.proj_up.weight]
        b = None
        if self.proj_up.bias is not None:
            b = torch.cat([self.proj_up_gate.bias, self.proj_up.bias])
        if ops.fused_linear_ok(x, ws):   # the bf16 image of the concatenation in one launch
            a = ops.fused_linear(x, ws, b)
        else:
            a = _linear(x, torch.cat(ws), b)
        if a.is_cuda and a.dtype == torch.bfloat16 and up % 4 == 0:
            # one HIP pass, one [dg | du] gradient
            return _linear(ops.swiglu(a), self.proj_down.weight, self.proj_down.bias)
        g, u = a.split([up, up], -1)
        return self.proj_down(F.silu(g) * u)


class mLSTMLayer(nn.Module):
    def __init__(self, cfg: xLSTMLargeConfig):
        super().__init__()
        self.cfg = cfg
        d = cfg.embedding_dim
        self.v_dim = int(d * cfg.v_dim_factor)
        self.qk_dim = int(d * cfg.qk_dim_factor)
        self.q = nn.Linear(d, self.qk_dim, bias=cfg.use_bias)
        self.k = nn.Linear(d, self.qk_dim, bias=cfg.use_bias)
        self.v = nn.Linear(d, self.v_dim, bias=cfg.use_bias)
        self.ogate_preact = nn.Linear(d, self.v_dim, bias=cfg.use_bias)
        self.igate_preact = nn.Linear(d, cfg.num_heads, bias=True)
        self.fgate_preact = nn.Linear(d, cfg.num_heads, bias=True)
        self.multihead_norm = MultiHeadLayerNorm(cfg.num_heads, self.v_dim // cfg.num_heads,
                                                 cfg.norm_eps, cfg.use_bias,
                                                 cfg.norm_reduction_force_float32)
        self.out_proj = nn.Linear(self.v_dim, d, bias=cfg.use_bias)

    def _mods(self):
        return (self.q, self.k, self.v, self.ogate_preact, self.igate_preact, self.fgate_preact)

    def projection(self, x):
        """[q | k | v | o | i | f] from ONE GEMM over the concatenated weight (the parameters and
        state_dict keep HF's six Linears): x is read and, under autocast, cast once instead of six
        times, and the two NH-wide gate projections (4 output columns each at C4) stop being
        GEMMs of their own."""
        mods = self._mods()
        ws = [m.weight for m in mods]
        b = None
        lead = 0   # leading bias columns that are cached zero pieces (no gradient to sum)
        if any(m.bias is not None for m in mods):
            b = torch.cat([m.bias if m.bias is not None else
                           _zeros(m.weight.shape[0], m.weight.dtype, m.weight.device)
                           for m in mods])
            for m in mods:
                if m.bias is not None:
                    break
                lead += m.weight.shape[0]
        if ops.fused_linear_ok(x, ws):   # the bf16 image of the concatenation in one launch
            return ops.fused_linear(x, ws, b, lead)
        return _linear(x, torch.cat(ws), b, lead)

    def projections(self, x):
        return self.projection(x).split([m.weight.shape[0] for m in self._mods()], -1)

    def forward(self, x, state=None):
        B, T, _ = x.shape
        NH = self.cfg.num_heads
        mh = self.multihead_norm
        kdt = getattr(torch, self.cfg.autocast_kernel_dtype)
        if x.is_cuda and mh.bias is None and mh.force_float32_reductions:
            a = self.projection(x)
            DQ, DV = self.qk_dim // NH, self.v_dim // NH
            if ops.mlstm_core_supported(a, NH, DQ, DV) and kdt in (torch.bfloat16, torch.float16):
                # split -> soft caps -> mLSTM cell -> gated head norm as one node reading q / k /
                # v / o in place from the projection (ops.MLSTMCoreFn); same math and roundings
                c0, n0, m0 = (None, None, None) if state is None else state
                y, c, n, m = ops.MLSTMCoreFn.apply(a, c0, n0, m0, mh.weight, NH, DQ, DV,
                                                   self.cfg.gate_soft_cap, self.cfg.eps, mh.eps, kdt)
                return _linear(y, self.out_proj.weight, self.out_proj.bias), (c, n, m)
            q, k, v, o, ig, fg = a.split([m.weight.shape[0] for m in self._mods()], -1)
        else:
            q, k, v, o, ig, fg = self.projections(x)
        # under autocast the cell runs in autocast_kernel_dtype (the reference passes float16,
        # model.py:227): q, k, v are cast to it as the xlstm fork's kernels cast their inputs.
        # Without autocast the activations' own dtype goes to the cell, as transformers' native
        # chunkwise cell (modeling_xlstm.py:323) ignores autocast_kernel_dtype; there is no fp32
        # HIP cell, so MLSTMFn computes fp32 activations in f16 (11-bit mantissa, the finer of
        # the compiled cells) whatever autocast_kernel_dtype says
        cell_dt = (kdt if x.is_cuda and torch.is_autocast_enabled("cuda")
                   and kdt in (torch.bfloat16, torch.float16) else q.dtype)
        q = q.reshape(B, T, NH, -1).transpose(1, 2).to(cell_dt)
        k = k.reshape(B, T, NH, -1).transpose(1, 2).to(cell_dt)
        v = v.reshape(B, T, NH, -1).transpose(1, 2).to(cell_dt)
        ig = soft_cap(ig, self.cfg.gate_soft_cap).transpose(1, 2)
        fg = soft_cap(fg, self.cfg.gate_soft_cap).transpose(1, 2)
        c0, n0, m0 = (None, None, None) if state is None else state
        h, new_state = mlstm_chunkwise(q, k, v, ig, fg, c0, n0, m0, return_last_states=True,
                                       eps=self.cfg.eps)
        mh = self.multihead_norm
        if h.dtype != o.dtype:
            h = h.to(o.dtype)   # the cell's output back to the step's activation dtype
        if (mh.bias is None and mh.force_float32_reductions and o.dtype == torch.bfloat16
                and ops.gated_head_norm_supported(h)):
            # sigmoid(o) * MultiHeadLayerNorm(h) in one HIP pass on the cell's [B,NH,T,DH] layout
            y = ops.gated_head_norm(h, o, mh.weight, mh.eps)
            return _linear(y, self.out_proj.weight, self.out_proj.bias), new_state
        h = self.multihead_norm(h.transpose(1, 2))
        return self.out_proj(torch.sigmoid(o) * h), new_state


def _add_norm(x, y, norm):
    """(x + y, norm(x + y)): the block's residual add and the RMSNorm that reads its result as
    one HIP pass (ops.AddRMSNormFn, bf16 roundings as the torch chain) where the glue kernels
    apply, else the torch chain itself."""
    if (isinstance(norm, RMSNorm) and norm.bias is None and norm.force_float32_reductions
            and x.shape == y.shape and ops.xlstm_glue_supported(x, x.shape[-1])
            and ops.xlstm_glue_supported(y, y.shape[-1])):
        return ops.add_rms_norm(x, y, norm.weight, norm.eps)
    s = x + y
    return s, norm(s)


class xLSTMBlock(nn.Module):
    def __init__(self, cfg: xLSTMLargeConfig):
        super().__init__()
        self.norm_mlstm = RMSNorm(cfg.embedding_dim, cfg.norm_eps, cfg.use_bias,
                                  cfg.norm_reduction_force_float32)
        self.mlstm_layer = mLSTMLayer(cfg)
        self.norm_ffn = RMSNorm(cfg.embedding_dim, cfg.norm_eps, cfg.use_bias,
                                cfg.norm_reduction_force_float32)
        self.ffn = FeedForward(cfg)

    def forward(self, x, state=None):
        y, state = self.mlstm_layer(self.norm_mlstm(x), state)
        x, n = _add_norm(x, y, self.norm_ffn)
        return x + self.ffn(n), state


class xLSTMLarge(nn.Module):
    """The encoder ASRModel builds for ``--encoder xlstm`` (model.py:301-307)."""

    def __init__(self, config: xLSTMLargeConfig):
        super().__init__()
        self.config = config
        d_in = config.input_dim if config.input_dim is not None else config.embedding_dim
        self.embedding = nn.Linear(d_in, config.embedding_dim)
        self.blocks = nn.ModuleList([xLSTMBlock(config) for _ in range(config.num_blocks)])
        self.out_norm = (RMSNorm(config.embedding_dim, config.norm_eps, config.use_bias,
                                 config.norm_reduction_force_float32)
                         if config.add_out_norm else nn.Identity())
        self.lm_head = nn.Linear(config.embedding_dim, config.vocab_size, bias=False)

    def forward(self, x, state=None):
        x = self.embedding(x)
        new_state = {}
        # xLSTMBlock.forward unrolled so that every residual add meets the RMSNorm reading its
        # result in one pass (_add_norm): the FFN branch of block i is added by block i+1's
        # norm_mlstm (or the output norm), the mLSTM branch by the block's own norm_ffn
        pending = None
        for i, blk in enumerate(self.blocks):
            if pending is None:
                n = blk.norm_mlstm(x)
            else:
                x, n = _add_norm(x, pending, blk.norm_mlstm)
            y, new_state[i] = blk.mlstm_layer(n, None if state is None else state.get(i))
            x, n = _add_norm(x, y, blk.norm_ffn)
            pending = blk.ffn(n)
        if pending is None:
            h = self.out_norm(x)
        else:
            x, h = _add_norm(x, pending, self.out_norm)
        logits = soft_cap(self.lm_head(h), self.config.output_logit_soft_cap)
        if self.config.return_last_states:
            return logits, new_state
        return logits
