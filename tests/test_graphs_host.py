"""CPU checks of graphs.GraphedSegments' preconditions (the capture itself needs the GPU:
tests/test_gpu_graphs.py).  A trainer it cannot capture faithfully is refused up front, before
any capture: DDP, gradient accumulation, an optimizer the HIP clip + Adam does not step, host
segments."""
import types

import pytest
import torch
import torch.nn as nn


def _trainer(**kw):
    from statecatcher_amd.train import SegmentTrainer
    model = nn.Linear(4, 4)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    return SegmentTrainer(model, nn.MSELoss(), opt, **kw)


def _segs():
    return [dict(feats=torch.zeros(1, 2, 4), masks=torch.ones(1, 2, dtype=torch.bool),
                 tokens=torch.zeros(1, 1, dtype=torch.long), in_lens=torch.tensor([2]),
                 tgt_lens=torch.tensor([1]))]


def test_refuses_gradient_accumulation():
    from statecatcher_amd.graphs import GraphedSegments
    with pytest.raises(ValueError, match="accumulation"):
        GraphedSegments(_trainer(accumulation_steps=2), _segs())


def test_refuses_an_optimizer_the_hip_adam_does_not_step():
    from statecatcher_amd.graphs import GraphedSegments
    tr = _trainer()   # CPU parameters: not eligible for the HIP clip + Adam
    with pytest.raises(ValueError, match="HIP clip"):
        GraphedSegments(tr, _segs())


def test_refuses_a_ddp_wrapped_trainer(monkeypatch):
    """A DDP-wrapped trainer is refused: DDP's reducer hooks sit on the gradient accumulators and
    would run inside the capture; under world > 1 the graphs broadcast and all-reduce themselves
    (build the trainer with ddp=False; tests/test_gpu_ddp.py pins it against eager DDP)."""
    from statecatcher_amd.graphs import GraphedSegments
    tr = _trainer()
    tr.ddp = True
    with pytest.raises(ValueError, match="ddp=False"):
        GraphedSegments(tr, _segs())


def test_refuses_host_segments(monkeypatch):
    from statecatcher_amd import graphs
    monkeypatch.setattr(graphs, "hip_adam_eligible", lambda opt: True)
    with pytest.raises(ValueError, match="device tensors"):
        graphs.GraphedSegments(_trainer(), _segs())
    with pytest.raises(ValueError, match="device tensors"):
        graphs.GraphedSegments(_trainer(), [])


def test_step_before_capture_raises(monkeypatch):
    from statecatcher_amd import graphs
    monkeypatch.setattr(graphs, "hip_adam_eligible", lambda opt: True)
    seg = _segs()[0]
    seg["feats"] = types.SimpleNamespace(is_cuda=True, device=torch.device("cpu"))
    gs = graphs.GraphedSegments(_trainer(), [seg])
    with pytest.raises(RuntimeError, match="before capture"):
        gs.step()


def test_refuses_periodic_checkpoints(monkeypatch, tmp_path):
    """save_every_n_updates is skipped by replay (step only replays and steps): refused up front
    instead of silently never saving."""
    from statecatcher_amd import graphs
    monkeypatch.setattr(graphs, "hip_adam_eligible", lambda opt: True)
    seg = _segs()[0]
    seg["feats"] = types.SimpleNamespace(is_cuda=True, device=torch.device("cpu"))
    tr = _trainer(save_every_n_updates=10, model_dir=str(tmp_path))
    with pytest.raises(ValueError, match="save_every_n_updates"):
        graphs.GraphedSegments(tr, [seg])
