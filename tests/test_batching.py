"""Segment batch assembly (statecatcher_amd/batching.py) against restated reference semantics
(train.py:186-212, :455-456, :478-487), on CPU: ragged segment counts under clipping and
padding, empty texts, blank padding of tokens, frame geometry."""
import pytest
import torch

from statecatcher_amd.batching import (frame_geometry, iterate_segments, prepare_batch_data,
                                       prepare_tokens_and_lengths, segment_count)

S = 480   # samples per segment


def ref_prepare_batch_data(audios_items, texts_items, masks_items, seg_idx, target_samples):
    """train.py:186-201, restated."""
    sa, sm, st = [], [], []
    for audios, texts, masks in zip(audios_items, texts_items, masks_items):
        if seg_idx < len(audios):
            sa.append(audios[seg_idx])
            sm.append(masks[seg_idx])
            st.append(texts[seg_idx])
        else:
            sa.append(torch.zeros(target_samples, dtype=torch.float32))
            sm.append(torch.zeros(target_samples, dtype=torch.bool))
            st.append("")
    return torch.stack(sa), torch.stack(sm), st


def ref_tokens(texts, encode, blank):
    """train.py:203-212, restated."""
    ids = [encode(t) for t in texts]
    lens = [len(t) for t in ids]
    tok = torch.full((len(ids), max(lens)), blank, dtype=torch.long)
    for i, t in enumerate(ids):
        if t:
            tok[i, :len(t)] = torch.tensor(t)
    return tok, lens


def encode(text):
    """A deterministic stand-in tokenizer: one id per character, in [1, 30]."""
    return [1 + (ord(c) % 30) for c in text]


def make_batch(counts, seed=0):
    g = torch.Generator().manual_seed(seed)
    A, T, M = [], [], []
    for i, n in enumerate(counts):
        A.append([torch.randn(S, generator=g) for _ in range(n)])
        M.append([torch.rand(S, generator=g) > 0.2 for _ in range(n)])
        T.append(["" if (i + k) % 4 == 0 else f"seg {i} {k} " * (k + 1) for k in range(n)])
    return A, T, M


@pytest.mark.parametrize("strategy,expect", [("clipping", 1), ("padding", 4)])
def test_segment_count_ragged(strategy, expect):
    assert segment_count([3, 1, 4, 2], strategy) == expect
    assert segment_count([], strategy) == 0
    with pytest.raises(ValueError):
        segment_count([1], "truncate")


@pytest.mark.parametrize("strategy", ["clipping", "padding"])
def test_slices_match_reference_semantics(strategy):
    A, T, M = make_batch([3, 1, 4, 2])
    seen = []
    for k, audio, mask, texts in iterate_segments(A, T, M, strategy, S, "cpu"):
        ra, rm, rt = ref_prepare_batch_data(A, T, M, k, S)
        assert torch.equal(audio, ra) and torch.equal(mask, rm) and texts == rt
        assert audio.dtype == torch.float32 and mask.dtype == torch.bool
        seen.append(k)
    assert seen == list(range(segment_count([3, 1, 4, 2], strategy)))


def test_missing_segments_are_zero_audio_false_mask_empty_text():
    A, T, M = make_batch([1, 3])
    audio, mask, texts = prepare_batch_data(A, T, M, 2, S, "cpu")
    assert not audio[0].any() and not mask[0].any() and texts[0] == ""
    assert torch.equal(audio[1], A[1][2]) and texts[1] == T[1][2]


def test_wrong_segment_size_is_an_error():
    A, T, M = make_batch([1])
    A[0][0] = torch.zeros(S - 1)
    with pytest.raises(ValueError):
        prepare_batch_data(A, T, M, 0, S, "cpu")


@pytest.mark.parametrize("texts", [["abc", "", "hello world"], ["", "x"], ["same", "same"]])
def test_tokens_blank_padded_like_reference(texts):
    tok, lens = prepare_tokens_and_lengths(texts, encode, blank_id=0, device="cpu")
    rtok, rlens = ref_tokens(texts, encode, 0)
    assert torch.equal(tok, rtok) and lens == rlens
    tok7, _ = prepare_tokens_and_lengths(texts, encode, blank_id=7, device="cpu")
    assert (tok7[0, lens[0]:] == 7).all()


def test_all_empty_texts_give_zero_width_tokens():
    tok, lens = prepare_tokens_and_lengths(["", ""], encode, 0, "cpu")
    assert tok.shape == (2, 0) and lens == [0, 0]


def test_frame_geometry_matches_reference():
    mask = torch.zeros(2, 1600, dtype=torch.bool)
    mask[0] = True
    mask[1, :1000] = True
    sub, fm, il = frame_geometry(mask, 10)
    assert sub == 160.0 and fm.shape == (2, 10)
    assert il.tolist() == [10, 6]
    sub2, fm2, il2 = frame_geometry(mask, 10, stack_order=2)
    assert sub2 == 320.0 and fm2.shape == (2, 5) and il2.tolist() == [5, 3]
