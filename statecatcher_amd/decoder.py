"""Drop-in of /root/reference/decoder.py:3-30 running on the GPU (one host copy, no per-frame sync)."""
import torch

from .ops import ctc_greedy_decode


def ctc_greedy_decoder(log_probs, input_lengths, blank=0):
    """log_probs [B,T,V], input_lengths [B] -> List[List[int]] (argmax, trim, collapse, drop blank)."""
    tokens, counts = ctc_greedy_decode(log_probs, input_lengths, blank)
    tokens = tokens.cpu()
    counts = counts.cpu().tolist()
    return [tokens[b, :c].tolist() for b, c in enumerate(counts)]
