"""Segment batch assembly of the reference training loop.

The reference cuts every utterance into fixed-size segments (dataset.py:179-262) and trains on
"segment slices": slice k stacks segment k of every batch item (train.py:186-201).  Items have
ragged segment counts; the batch runs K slices with K = min(counts) under the "clipping"
strategy and K = max(counts) under "padding", where an item that has run out contributes a zero
audio segment, an all-false sample mask and an empty text (train.py:455-456, :192-195).  Texts
become blank-padded token rows (train.py:203-212).

Same semantics here, with the host->device traffic shaped for the GPU: a slice is stacked into
one pinned host buffer and crosses PCIe as ONE non-blocking copy (the reference copies per item
and per token row, train.py:199-200, :211), and the token matrix is built on the host and copied
once.  Frame masks / input lengths follow train.py:478-487 (``frame_geometry``).
"""
from typing import Callable, List, Sequence, Tuple

import torch

from .train import compute_frame_mask

STRATEGIES = ("clipping", "padding")


def segment_count(seg_counts: Sequence[int], strategy: str) -> int:
    """Number of segment slices in a batch (train.py:455-456)."""
    if strategy not in STRATEGIES:
        raise ValueError(f"batch_segment_strategy must be one of {STRATEGIES}, got {strategy!r}")
    if not seg_counts:
        return 0
    return min(seg_counts) if strategy == "clipping" else max(seg_counts)


def _to_device(host: torch.Tensor, device) -> torch.Tensor:
    dev = torch.device(device)
    if dev.type == "cpu":
        return host
    return host.to(dev, non_blocking=True)


def prepare_batch_data(batch_audio_items, batch_texts_items, batch_masks_items, seg_idx: int,
                       target_samples: int, device):
    """Slice ``seg_idx`` of the batch (train.py:186-201): per item its segment ``seg_idx``, or
    zeros / an all-false mask / "" when the item has fewer segments.  Returns (audio [B, S] fp32,
    mask [B, S] bool, texts).  Each segment must hold exactly ``target_samples`` samples (the
    dataset pads/trims to it, dataset.py:221-262)."""
    B = len(batch_audio_items)
    pin = torch.device(device).type == "cuda"
    audio = torch.zeros(B, target_samples, dtype=torch.float32, pin_memory=pin)
    mask = torch.zeros(B, target_samples, dtype=torch.bool, pin_memory=pin)
    texts: List[str] = []
    for i, (audios, txts, masks) in enumerate(zip(batch_audio_items, batch_texts_items,
                                                  batch_masks_items)):
        if seg_idx < len(audios):
            a, m = audios[seg_idx], masks[seg_idx]
            if a.numel() != target_samples or m.numel() != target_samples:
                raise ValueError(f"item {i} segment {seg_idx}: {a.numel()} samples / {m.numel()} "
                                 f"mask entries, expected {target_samples}")
            audio[i].copy_(a.reshape(-1))
            mask[i].copy_(m.reshape(-1))
            texts.append(txts[seg_idx])
        else:
            texts.append("")
    return _to_device(audio, device), _to_device(mask, device), texts


def prepare_tokens_and_lengths(slice_texts: Sequence[str], encode: Callable[[str], List[int]],
                               blank_id: int, device) -> Tuple[torch.Tensor, List[int]]:
    """train.py:203-212: token ids per text, padded with ``blank_id`` to the longest -> (tokens
    [B, U_max] int64, target lengths).  ``encode`` maps a text to token ids (the reference calls
    sentencepiece's ``sp.encode(txt, out_type=int)``; pass ``sp.encode`` or any callable).  An
    all-empty slice gives a [B, 0] matrix, as the reference's max() of zero lengths does."""
    ids = [list(encode(t)) for t in slice_texts]
    lens = [len(t) for t in ids]
    umax = max(lens) if lens else 0
    pin = torch.device(device).type == "cuda"
    tokens = torch.full((len(ids), umax), blank_id, dtype=torch.long, pin_memory=pin)
    for i, t in enumerate(ids):
        if t:
            tokens[i, :len(t)] = torch.as_tensor(t, dtype=torch.long)
    return _to_device(tokens, device), lens


def frame_geometry(sample_mask: torch.Tensor, n_frames: int, stack_order: int = 1):
    """train.py:478-487: subsample = samples per frame x stack order, the frame mask and the
    CTC input lengths (floor(valid samples / subsample), clamped to the frame count)."""
    subsample = sample_mask.size(1) / n_frames * float(stack_order)
    frame_mask = compute_frame_mask(sample_mask, subsample)
    in_lens = (sample_mask.sum(dim=1) / subsample).clamp(max=n_frames).long()
    return subsample, frame_mask, in_lens


def iterate_segments(batch_audio_items, batch_texts_items, batch_masks_items, strategy: str,
                     target_samples: int, device):
    """Yields (seg_idx, audio, mask, texts) for the K slices of one server batch (train.py:455-466);
    the caller resets its encoder state before the first (train.py:460)."""
    K = segment_count([len(a) for a in batch_audio_items], strategy)
    for k in range(K):
        yield (k,) + prepare_batch_data(batch_audio_items, batch_texts_items, batch_masks_items, k,
                                        target_samples, device)
