"""Host logic of the data-parallel segment-carry loop (statecatcher_amd/train.py), on CPU.

world_size-2 gloo processes, each training its own batch shard with its own carried state,
must end with identical parameters, equal to one process training the whole batch (DDP
averages the per-rank mean-reduced CTC gradients = the global mean; clipping runs after the
all-reduce).  The encoder here is a small pure-torch stand-in with the ASRModel call signature
(the HIP encoder has no CPU path by design); what is under test is the loop: state carry,
accumulation with no_sync, clip, step, checkpoint format.
"""
import multiprocessing as mp
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.nn as nn

from statecatcher_amd.train import (SegmentTrainer, compute_frame_mask, frame_lengths,
                                    load_checkpoint, save_checkpoint)

B, T, F, H, V, SEGS, BATCHES = 4, 12, 6, 8, 7, 3, 2


class TinyStateful(nn.Module):
    """feats [B,T,F], mask, states -> (logits [B,T,V], states); states = ([h [B,H]], [s [B,H]])
    carried like LucyRNNtriton's (linear recurrence so the carry matters)."""

    def __init__(self):
        super().__init__()
        self.inp = nn.Linear(F, H)
        self.dec = nn.Parameter(torch.full((H,), 0.7))
        self.out = nn.Linear(H, V)

    def forward(self, feats, mask, states=None):
        x = self.inp(feats * mask.unsqueeze(-1).to(feats.dtype))
        h = states[0][0] if states is not None else torch.zeros(feats.shape[0], H)
        hs = []
        for t in range(x.shape[1]):
            h = torch.sigmoid(self.dec) * h + x[:, t]
            hs.append(h)
        y = torch.stack(hs, 1)
        return self.out(torch.tanh(y)), ([h], [h * 0.5])


def data(seed):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(BATCHES):
        segs = []
        for _ in range(SEGS):
            feats = torch.randn(B, T, F, generator=g)
            U = torch.randint(1, 4, (B,), generator=g)
            tok = torch.randint(1, V, (B, 3), generator=g)
            for b in range(B):
                tok[b, U[b]:] = 0
            segs.append((feats, torch.ones(B, T, dtype=torch.bool), tok, [T] * B, U.tolist()))
        out.append(segs)
    return out


def train(rank, world, accum, shard):
    torch.manual_seed(0)
    model = TinyStateful()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    tr = SegmentTrainer(model, nn.CTCLoss(blank=0, zero_infinity=True), opt,
                        accumulation_steps=accum, max_grad_norm=0.5, bucket_cap_mb=0.001)
    lo, hi = (rank * B // world, (rank + 1) * B // world) if shard else (0, B)
    losses = []
    for segs in data(1):
        tr.begin_batch()
        for feats, mask, tok, il, tl in segs:
            loss = tr.train_segment(feats[lo:hi], mask[lo:hi], tok[lo:hi], il[lo:hi], tl[lo:hi])
            losses.append(float(loss.detach()))
    return {k: v.detach().clone() for k, v in model.state_dict().items()}, losses


def _worker(rank, world, port, accum, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd, losses = train(rank, world, accum, shard=True)
        q.put((rank, {k: v.numpy() for k, v in sd.items()}, losses))   # by value, not by fd
    finally:
        dist.destroy_process_group()


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("accum", [1, 2])
def test_ddp_world2_matches_single_process_full_batch(accum):
    ctx = mp.get_context("spawn")   # fork after torch started its thread pools can deadlock
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, accum, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, sd, losses = q.get(timeout=120)
        res[rank] = ({k: torch.from_numpy(v) for k, v in sd.items()}, losses)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_sd, ref_losses = train(0, 1, accum, shard=False)
    for k in ref_sd:
        torch.testing.assert_close(res[0][0][k], res[1][0][k], rtol=0, atol=0)   # ranks agree bitwise
        torch.testing.assert_close(res[0][0][k], ref_sd[k], rtol=1e-5, atol=1e-6)
    # per-rank losses average to the full-batch loss (mean reduction, equal shards)
    for a, b, r in zip(res[0][1], res[1][1], ref_losses):
        assert abs((a + b) / 2 - r) < 1e-5 * max(1.0, abs(r))


def test_state_carry_resets_per_batch_and_feeds_next_segment():
    torch.manual_seed(0)
    model = TinyStateful()
    seen = []
    orig = model.forward

    def spy(feats, mask, states=None):
        seen.append(states)
        return orig(feats, mask, states)
    model.forward = spy
    tr = SegmentTrainer(model, nn.CTCLoss(zero_infinity=True), torch.optim.SGD(model.parameters(), lr=0.1))
    for segs in data(2):
        tr.begin_batch()
        for feats, mask, tok, il, tl in segs:
            tr.train_segment(feats, mask, tok, il, tl)
    assert seen[0] is None and seen[SEGS] is None           # reset at every batch
    assert seen[1] is not None and not seen[1][0][0].requires_grad   # carried, detached
    assert tr.global_step == SEGS * BATCHES


def test_checkpoint_roundtrip_reference_format(tmp_path):
    torch.manual_seed(0)
    m = TinyStateful()
    path = save_checkpoint(str(tmp_path), m, None, epoch=0, global_step=7)
    assert os.path.basename(path) == "model_epoch1_step7.pt"
    ck = torch.load(path, weights_only=True)
    assert set(ck) == {"model"} and set(ck["model"]) == set(m.state_dict())
    m2 = TinyStateful()
    with torch.no_grad():
        for p in m2.parameters():
            p.zero_()
    load_checkpoint(path, m2)
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k])


def test_frame_mask_and_lengths_match_reference_semantics():
    mask = torch.zeros(2, 1600, dtype=torch.bool)
    mask[0, :1600] = True
    mask[1, :1000] = True
    fm = compute_frame_mask(mask, 160.0)
    assert fm.shape == (2, 10)
    assert fm[0].all() and fm[1, :7].all() and not fm[1, 7:].any()   # frame 6 partially covered
    assert frame_lengths(mask, 160.0, 10) == [10, 6]                  # floor(1000/160) = 6


class TorchRNNTLoss(nn.Module):
    """warp_rnnt's keyword interface (model.py:97-105) over a tiny differentiable torch lattice
    (test stand-in: the product loss is HIP-only)."""

    def forward(self, log_probs, labels, frames_lengths, labels_lengths, blank_id=0, compact=False,
                gather=True):
        nll = []
        for b in range(log_probs.shape[0]):
            Tb, Ub = int(frames_lengths[b]), int(labels_lengths[b])
            lp = log_probs[b]
            alpha = [[None] * (Ub + 1) for _ in range(Tb)]
            for t in range(Tb):
                for u in range(Ub + 1):
                    terms = []
                    if t == 0 and u == 0:
                        terms.append(lp.new_zeros(()))
                    if t > 0:
                        terms.append(alpha[t - 1][u] + lp[t - 1, u, blank_id])
                    if u > 0:
                        terms.append(alpha[t][u - 1] + lp[t, u - 1, labels[b, u - 1]])
                    alpha[t][u] = torch.logsumexp(torch.stack(terms), 0)
            nll.append(-(alpha[Tb - 1][Ub] + lp[Tb - 1, Ub, blank_id]))
        return torch.stack(nll).mean()


def test_rnnt_segment_through_trainer_saves_joiner_and_skips_joiner_clip(tmp_path):
    from statecatcher_amd.model import RNNTPredictorJoiner
    torch.manual_seed(0)
    model = TinyStateful()
    joiner = RNNTPredictorJoiner(V, 4, 6, V)
    opt = torch.optim.Adam(list(model.parameters()) + list(joiner.parameters()), lr=1e-2)
    with pytest.raises(ValueError):
        SegmentTrainer(model, TorchRNNTLoss(), opt, mode="rnnt")
    tr = SegmentTrainer(model, TorchRNNTLoss(), opt, mode="rnnt", joiner=joiner, max_grad_norm=1e-3,
                        save_every_n_updates=1, model_dir=str(tmp_path))
    assert not tr._fused_clip_ok()   # the joiner is in the optimizer: clip model params only
    j0 = {k: v.clone() for k, v in joiner.state_dict().items()}
    feats, mask, tok, il, tl = data(3)[0][0]
    loss = tr.train_segment(feats, mask, tok, il, tl)
    assert torch.isfinite(loss)
    assert any(not torch.equal(j0[k], v) for k, v in joiner.state_dict().items())   # joiner trained
    ck = torch.load(os.path.join(tmp_path, "model_epoch1_step1.pt"), weights_only=True)
    assert set(ck) == {"model", "joiner"} and set(ck["joiner"]) == set(joiner.state_dict())


def train_rnnt(rank, world, shard):
    """C5's loop shape: the encoder AND the joiner DDP-wrapped (train.py:368-375 puts both in one
    optimizer), clip over the encoder's parameters only."""
    from statecatcher_amd.model import RNNTPredictorJoiner
    torch.manual_seed(0)
    model = TinyStateful()
    joiner = RNNTPredictorJoiner(V, 4, 6, V)
    opt = torch.optim.Adam(list(model.parameters()) + list(joiner.parameters()), lr=1e-2)
    tr = SegmentTrainer(model, TorchRNNTLoss(), opt, mode="rnnt", joiner=joiner, max_grad_norm=0.5,
                        bucket_cap_mb=0.001)
    if world > 1:
        assert isinstance(tr.joiner_net, nn.parallel.DistributedDataParallel)
    lo, hi = (rank * B // world, (rank + 1) * B // world) if shard else (0, B)
    losses = []
    for segs in data(2)[:1]:
        tr.begin_batch()
        for feats, mask, tok, il, tl in segs[:2]:
            loss = tr.train_segment(feats[lo:hi], mask[lo:hi], tok[lo:hi], il[lo:hi], tl[lo:hi])
            losses.append(float(loss.detach()))
    sd = {f"m.{k}": v.detach().clone() for k, v in model.state_dict().items()}
    sd.update({f"j.{k}": v.detach().clone() for k, v in joiner.state_dict().items()})
    return sd, losses


def _worker_rnnt(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd, losses = train_rnnt(rank, world, shard=True)
        q.put((rank, {k: v.numpy() for k, v in sd.items()}, losses))
    finally:
        dist.destroy_process_group()


def test_rnnt_ddp_world2_matches_single_process_full_batch():
    """The C5 (RNN-T) loop at world size 2: encoder and joiner both all-reduced, ranks bitwise
    equal, and equal to one process on the full batch (mean-reduced loss over equal shards)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker_rnnt, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, sd, losses = q.get(timeout=180)
        res[rank] = ({k: torch.from_numpy(v) for k, v in sd.items()}, losses)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_sd, ref_losses = train_rnnt(0, 1, shard=False)
    assert any(k.startswith("j.") for k in ref_sd)
    for k in ref_sd:
        torch.testing.assert_close(res[0][0][k], res[1][0][k], rtol=0, atol=0)
        torch.testing.assert_close(res[0][0][k], ref_sd[k], rtol=1e-5, atol=1e-6)
    for a, b, r in zip(res[0][1], res[1][1], ref_losses):
        assert abs((a + b) / 2 - r) < 1e-5 * max(1.0, abs(r))


class TinyDictStateful(TinyStateful):
    """The xLSTM encoder's state shape (C4): a dict of per-block tuples, carried the same way."""

    def forward(self, feats, mask, states=None):
        prev = None if states is None else ([states["block0"][0]], None)
        logits, (hs, _) = super().forward(feats, mask, prev)
        return logits, {"block0": (hs[0], hs[0] * 0.25, torch.zeros(feats.shape[0], 1))}


def train_dict(rank, world, shard):
    torch.manual_seed(0)
    model = TinyDictStateful()
    opt = torch.optim.Adam(model.parameters(), lr=1e-2)
    tr = SegmentTrainer(model, nn.CTCLoss(blank=0, zero_infinity=True), opt, max_grad_norm=0.5,
                        bucket_cap_mb=0.001)
    lo, hi = (rank * B // world, (rank + 1) * B // world) if shard else (0, B)
    losses = []
    for segs in data(4):
        tr.begin_batch()
        for feats, mask, tok, il, tl in segs:
            losses.append(float(tr.train_segment(feats[lo:hi], mask[lo:hi], tok[lo:hi], il[lo:hi],
                                                 tl[lo:hi]).detach()))
            assert isinstance(tr.encoder_state, dict)
    return {k: v.detach().clone() for k, v in model.state_dict().items()}, losses


def _worker_dict(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sd, losses = train_dict(rank, world, shard=True)
        q.put((rank, {k: v.numpy() for k, v in sd.items()}, losses))
    finally:
        dist.destroy_process_group()


def test_dict_state_ddp_world2_matches_single_process_full_batch():
    """C4's loop shape (dict-of-tuples encoder state, as xLSTMLarge returns) at world size 2."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker_dict, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        rank, sd, losses = q.get(timeout=120)
        res[rank] = ({k: torch.from_numpy(v) for k, v in sd.items()}, losses)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_sd, ref_losses = train_dict(0, 1, shard=False)
    for k in ref_sd:
        torch.testing.assert_close(res[0][0][k], res[1][0][k], rtol=0, atol=0)
        torch.testing.assert_close(res[0][0][k], ref_sd[k], rtol=1e-5, atol=1e-6)
    for a, b, r in zip(res[0][1], res[1][1], ref_losses):
        assert abs((a + b) / 2 - r) < 1e-5 * max(1.0, abs(r))
