"""Oracle (TEST INFRASTRUCTURE ONLY): CTC greedy decoding, integer path.

Restates /root/reference/decoder.py:3-30: argmax over V (first index of the maximum, as
``torch.argmax`` returns; a NaN counts as the maximum), trim to ``input_lengths[b]``,
collapse repeats, drop blank.
"""
import numpy as np


def argmax_first(x):
    """torch.argmax semantics on the last axis: first max; NaN wins (first NaN)."""
    x = np.asarray(x)
    nan = np.isnan(x)
    idx = np.argmax(x, axis=-1)            # numpy: first occurrence of max, NaN propagates
    has_nan = nan.any(axis=-1)
    first_nan = np.argmax(nan, axis=-1)
    return np.where(has_nan, first_nan, idx)


def ctc_greedy(log_probs, input_lengths, blank=0):
    preds = argmax_first(log_probs)        # decoder.py:16
    out = []
    for b in range(preds.shape[0]):
        prev = None
        seq = []
        for tok in preds[b, : int(input_lengths[b])]:   # decoder.py:20-27
            tok = int(tok)
            if tok != blank and tok != prev:
                seq.append(tok)
            prev = tok
        out.append(seq)
    return out
