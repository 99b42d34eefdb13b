"""The callers of the hot path, with the reference's signatures (model.py:11-110, :282-398).

`compute_loss` / `ASRModel` / `detach_states` keep /root/reference/model.py's call pattern so
the reference train.py segment loop drives them unchanged.  Only the LucyRNN encoders are
built here (the hot path); the CTC branch runs the fused HIP CTC when the criterion is
statecatcher_amd.model.CTCLoss and otherwise exactly the reference's
`log_softmax -> transpose -> criterion` sequence.
"""
from typing import Any, Optional

import torch
import torch.nn as nn

from .lucyrnn_conf import LucyRNNConfig
from .lucyrnn_triton import LucyRNNtriton
from .ops import ctc_loss


def detach_states(states):
    """Recursively detach tensors in nested dict/tuple/list states (model.py:11-25)."""
    if states is None:
        return None
    if isinstance(states, torch.Tensor):
        return states.detach()
    if isinstance(states, dict):
        return {k: detach_states(v) for k, v in states.items()}
    if isinstance(states, tuple):
        return tuple(detach_states(s) for s in states)
    if isinstance(states, list):
        return [detach_states(s) for s in states]
    return states


def assert_all_detached(x):
    """model.py:27-35."""
    if isinstance(x, torch.Tensor):
        assert not x.requires_grad, "Tensor still requires grad"
    elif isinstance(x, (list, tuple)):
        for v in x:
            assert_all_detached(v)
    elif isinstance(x, dict):
        for v in x.values():
            assert_all_detached(v)


class CTCLoss(nn.Module):
    """nn.CTCLoss(blank, reduction, zero_infinity) on the HIP alpha-beta kernels.

    forward(log_probs [T,B,V], targets [B,U], input_lengths, target_lengths) follows
    nn.CTCLoss's interface (train.py:142); forward_logits(logits [B,T,V], ...) fuses the
    log_softmax that model.py:70 applies first and skips the transpose.
    """

    def __init__(self, blank=0, reduction="mean", zero_infinity=True):
        super().__init__()
        self.blank = blank
        self.reduction = reduction
        self.zero_infinity = zero_infinity

    def forward(self, log_probs, targets, input_lengths, target_lengths):
        return ctc_loss(log_probs.transpose(0, 1), targets, input_lengths, target_lengths,
                        blank=self.blank, reduction=self.reduction,
                        zero_infinity=self.zero_infinity, is_logits=False)

    def forward_logits(self, logits, targets, input_lengths, target_lengths):
        return ctc_loss(logits, targets, input_lengths, target_lengths, blank=self.blank,
                        reduction=self.reduction, zero_infinity=self.zero_infinity,
                        is_logits=True)


def compute_loss(mode: str, criterion: nn.Module, model: nn.Module, feats: torch.Tensor,
                 masks: torch.Tensor, tokens: torch.Tensor, in_lens, tgt_lens, blank_id: int,
                 use_rnnt_joiner: Optional[nn.Module] = None, input_state: Optional[Any] = None,
                 args=None, compact=False):
    """model.py:37-110: returns (loss, output_state, enc_out, output_state)."""
    if input_state:
        input_state = detach_states(input_state)
        if args is not None and getattr(args, "debug", False):
            assert_all_detached(input_state)
    enc_out, output_state = model(feats, masks, input_state)
    if mode == "ctc":
        if isinstance(criterion, CTCLoss):
            loss = criterion.forward_logits(enc_out, tokens, in_lens, tgt_lens)
        else:
            logp = enc_out.log_softmax(-1).transpose(0, 1)
            loss = criterion(logp, tokens, in_lens, tgt_lens)
    elif mode == "rnnt":
        raise NotImplementedError("RNN-T loss kernels are not built yet (SURVEY §8a a11, next row)")
    else:
        raise ValueError(f"Unknown mode: {mode}")
    return loss, output_state, enc_out, output_state


class ASRModel(nn.Module):
    """model.py:282-398, LucyRNN branch: optional input projection, zero-masking of padded
    frames, encoder call with/without carried state."""

    def __init__(self, frontend: Optional[nn.Module], encoder, vocab_size: int, feat_dim: int,
                 proj_dim: int, debug: bool = False):
        super().__init__()
        self.frontend = frontend
        self.debug = debug
        if isinstance(encoder, LucyRNNConfig):
            self.cfg = encoder
            self.encoder = LucyRNNtriton(self.cfg)
            self.enc_out_dim = vocab_size
            self.input_seq_pad_factor = 8
            if proj_dim > 0:
                self.proj = nn.Linear(feat_dim, proj_dim)
        else:
            raise ValueError(f"Unknown encoder provided: {type(encoder)}")

    def forward(self, feats, mask, states=None):
        if hasattr(self, "proj"):
            feats = self.proj(feats)
        if mask is not None:
            feats = feats * mask.unsqueeze(-1).to(feats.dtype)
        if states is not None:
            logits, new_states = self.encoder(feats, states)
        else:
            logits, new_states = self.encoder(feats)
        return logits, new_states


def build_lucyrnn_config(input_dim, hidden_size, num_layers, vocab_size, is_training=True):
    """model.py:231-245: the LucyRNN config train.py builds (triton kernel, fused ops, no LN)."""
    return LucyRNNConfig(input_dim=input_dim, hidden_dim=hidden_size, num_layers=num_layers,
                         vocab_size=vocab_size, return_last_states=True, kernel_impl="triton",
                         fused_ops=True, stack_order=1, layer_norm=False, is_training=is_training)
