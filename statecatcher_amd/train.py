"""The reference's segment-carry training loop around the hot path, data-parallel.

Mirrors /root/reference/train.py:
  * ``compute_frame_mask``      train.py:296-306 (sample mask -> frame mask)
  * ``frame_lengths``           train.py:486-487 (in_lens from the sample mask)
  * ``save_checkpoint``         train.py:267-283 ({"model": state_dict[, "joiner": ...]})
  * ``SegmentTrainer``          train.py:460-581: per server batch the encoder state starts
    empty; per segment compute_loss with the carried (detached) state, loss / accumulation
    steps, backward, and every ``accumulation_steps`` segments clip_grad_norm_ + optimizer
    step + zero_grad; the segment's output state becomes the next input state.

Data parallel (new; the reference is single-process): when torch.distributed is
initialised with world size > 1 the model is wrapped in DistributedDataParallel (one process
per GPU, backend "nccl" = RCCL over xGMI; "gloo" in the CPU tests).  Each rank trains its own
batch shard and carries its own encoder state; gradients are all-reduced in buckets overlapped
with the backward, and only on the segments that step the optimizer (``no_sync`` on the
accumulation-only ones).  Clipping runs after the all-reduce, so every rank applies the same
update.  Checkpoints hold the unwrapped module's state_dict, keys unchanged.
"""
import contextlib
import os
from typing import Any, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from .model import compute_loss
from .optim import clip_and_adam_step, hip_adam_eligible


def compute_frame_mask(sample_mask: torch.Tensor, subsample: float) -> torch.Tensor:
    """[B, S] sample mask -> [B, T] frame mask, T = int(S / subsample) (train.py:296-306)."""
    B, S = sample_mask.shape
    T = int(S / subsample)
    S_trim = S - (S % T)
    reshaped = sample_mask[:, :S_trim].reshape(B, T, int(subsample))
    return reshaped.any(dim=2)


def frame_lengths(sample_mask: torch.Tensor, subsample: float, T: int):
    """CTC input lengths as the reference computes them (train.py:486-487)."""
    return (sample_mask.sum(dim=1) / subsample).clamp(max=T).long().tolist()


def unwrap(model: nn.Module) -> nn.Module:
    return model.module if isinstance(model, nn.parallel.DistributedDataParallel) else model


def save_checkpoint(model_dir, model, joiner, epoch, global_step=None):
    """train.py:267-283: file name and payload as the reference writes them."""
    name = f"model_epoch{epoch + 1}_step{global_step}.pt" if global_step is not None \
        else f"model_epoch{epoch + 1}.pt"
    path = os.path.join(model_dir, name)
    torch.save({"model": unwrap(model).state_dict(),
                **({"joiner": unwrap(joiner).state_dict()} if joiner is not None else {})}, path)
    return path


def load_checkpoint(path, model, joiner=None, map_location="cpu"):
    """Loads a reference-format checkpoint (tensors only: weights_only=True)."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    unwrap(model).load_state_dict(ck["model"])
    if joiner is not None and "joiner" in ck:
        unwrap(joiner).load_state_dict(ck["joiner"])
    return ck


class SegmentTrainer:
    """One trainer per rank.  ``begin_batch()`` at every new server batch, then
    ``train_segment(...)`` per segment, exactly in train.py's order."""

    def __init__(self, model: nn.Module, criterion: nn.Module, optimizer, mode: str = "ctc",
                 blank_id: int = 0, accumulation_steps: int = 1, max_grad_norm: float = 50.0,
                 amp_dtype: Optional[torch.dtype] = None, bucket_cap_mb: float = 50.0,
                 save_every_n_updates: Optional[int] = None, model_dir: Optional[str] = None,
                 joiner: Optional[nn.Module] = None, compact_rnnt: bool = False,
                 ddp: Optional[bool] = None):
        if mode == "rnnt" and joiner is None:
            raise ValueError("mode='rnnt' needs the joiner module (train.py:144-146 builds it)")
        self.model = model
        self.joiner = joiner
        self.compact_rnnt = compact_rnnt
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        # ddp=None: wrap whenever the job has more than one rank; True: wrap at any world size
        # (an initialised process group is required), e.g. a 1-rank RCCL group
        self.ddp = self.world > 1 if ddp is None else bool(ddp)
        if self.ddp and not (dist.is_available() and dist.is_initialized()):
            raise ValueError("ddp=True needs an initialised torch.distributed process group")
        if self.ddp:
            dev = next(model.parameters()).device
            self.net = nn.parallel.DistributedDataParallel(
                model, device_ids=[dev.index] if dev.type == "cuda" else None,
                bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
                broadcast_buffers=False)
            self.joiner_net = None if joiner is None else nn.parallel.DistributedDataParallel(
                joiner, device_ids=[dev.index] if dev.type == "cuda" else None,
                bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
                broadcast_buffers=False)
        else:
            self.net = model
            self.joiner_net = joiner
        self.criterion = criterion
        self.optimizer = optimizer
        self.mode = mode
        self.blank_id = blank_id
        self.accumulation_steps = max(1, int(accumulation_steps))
        self.max_grad_norm = max_grad_norm
        self.amp_dtype = amp_dtype
        self.save_every_n_updates = save_every_n_updates
        self.model_dir = model_dir
        self.global_step = 0
        self.epoch = 0
        self.encoder_state: Optional[Any] = None

    def _fused_clip_ok(self) -> bool:
        """The clip coefficient may ride on the fused Adam kernel only when every parameter the
        optimizer steps is one clip_grad_norm_ covers: the reference clips model.parameters()
        alone (train.py:553), so e.g. an RNN-T joiner in the same optimizer stays unscaled."""
        opt = self.optimizer
        if not (isinstance(opt, (torch.optim.Adam, torch.optim.AdamW))
                and all(g.get("fused") for g in opt.param_groups)
                and getattr(opt, "found_inf", None) is None):
            return False
        own = {id(p) for p in self.model.parameters()}
        return all(id(p) in own for g in opt.param_groups for p in g["params"])

    def _clip_and_step(self):
        """clip_grad_norm_(max_norm) then optimizer.step() (train.py:543-552).  A torch Adam /
        AdamW built as the reference builds it runs on HIP (optim.clip_and_adam_step).  With a fused
        Adam the clip coefficient is handed to the optimizer kernel as its gradient divisor
        (grads / max(1, (norm + 1e-6) / max_norm)), which equals clip_grad_norm_'s in-place
        scaling followed by the step, without the extra pass over every gradient."""
        params = [p for p in self.model.parameters() if p.grad is not None]
        if params and params[0].grad.is_cuda and hip_adam_eligible(self.optimizer):
            # the reference's Adam / AdamW: clip + step as two HIP launches (optim.py)
            clip_and_adam_step(self.optimizer, params, self.max_grad_norm)
            return
        if not (self._fused_clip_ok() and params and params[0].grad.is_cuda):
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.max_grad_norm)
            self.optimizer.step()
            return
        total = torch.nn.utils.get_total_norm([p.grad for p in params], 2.0)
        self.optimizer.grad_scale = torch.clamp((total + 1e-6) / self.max_grad_norm, min=1.0) \
            .to(torch.float32)
        try:
            self.optimizer.step()
        finally:
            self.optimizer.grad_scale = None

    def begin_batch(self):
        """New server batch: the carried encoder state starts empty (train.py:460)."""
        self.encoder_state = None

    def _steps_now(self) -> bool:
        return (self.global_step + 1) % self.accumulation_steps == 0

    def forward_backward(self, feats, masks, tokens, in_lens, tgt_lens, input_state):
        """compute_loss under the trainer's autocast + backward of loss / accumulation_steps
        (train.py:508-537) from ``input_state``.  Returns (loss, output_state).  No host sync:
        graphs.GraphedSegments captures this call as one HIP graph."""
        with torch.autocast(feats.device.type, dtype=self.amp_dtype or torch.float32,
                            enabled=self.amp_dtype is not None):
            loss, output_state, _, _ = compute_loss(
                self.mode, self.criterion, self.net, feats, masks, tokens, in_lens, tgt_lens,
                self.blank_id, use_rnnt_joiner=self.joiner_net, input_state=input_state,
                compact=self.compact_rnnt)
        # loss / accumulation_steps (train.py:535); a division by 1 is the identity
        (loss / self.accumulation_steps if self.accumulation_steps != 1 else loss).backward()
        return loss, output_state

    def train_segment(self, feats, masks, tokens, in_lens, tgt_lens):
        """One segment (train.py:508-581).  Returns the (un-divided) loss tensor."""
        stepping = self._steps_now()
        sync = contextlib.ExitStack()
        if not (stepping or not self.ddp):
            sync.enter_context(self.net.no_sync())
            if self.joiner_net is not None:
                sync.enter_context(self.joiner_net.no_sync())
        with sync:
            loss, output_state = self.forward_backward(feats, masks, tokens, in_lens, tgt_lens,
                                                       self.encoder_state)
        if stepping:
            self._clip_and_step()
            self.optimizer.zero_grad(set_to_none=True)
        if self.save_every_n_updates and (self.global_step + 1) % self.save_every_n_updates == 0 \
                and (self.world == 1 or dist.get_rank() == 0) and self.model_dir:
            # train.py:576-578: the joiner is saved alongside the model in RNN-T mode
            save_checkpoint(self.model_dir, self.model, self.joiner if self.mode == "rnnt" else None,
                            self.epoch, self.global_step + 1)
        self.encoder_state = output_state
        self.global_step += 1
        return loss
