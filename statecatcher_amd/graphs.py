"""The segment loop's forward + backward replayed as HIP graphs (one per segment position).

The reference's training loop (/root/reference/train.py:460-581) runs, per segment, compute_loss
with the carried state, backward, clip + Adam.  On MI355X the forward + backward of one segment
is ~90 kernel launches; the host issues them in ~2.8 ms against a ~5 ms GPU step
(DESIGN.md §6 item 7), so the host is one halving of the GPU step away from being the bound.
``GraphedSegments`` captures ``SegmentTrainer.forward_backward`` of a FIXED list of
device-resident segments once, one graph per position in the server batch (one shared memory
pool), and replays them:

  * graph 0 starts the batch (no input state, train.py:460); graph i > 0 reads graph i - 1's
    output state in place, so replaying 0, 1, ..., n - 1 is the eager loop's state chain;
  * each graph rebuilds the bf16 weight images it reads (ops.weight_images, inside the graph),
    so it always sees the weights of the optimizer step before it;
  * the gradients each graph writes are its own static tensors: after a replay they become the
    parameters' ``.grad`` and the clip + Adam step (optim.clip_and_adam_step, 3-4 launches) runs
    eagerly, as in ``SegmentTrainer.train_segment``.

Same kernels in the same order as the eager step, so the losses and weights are bitwise the
eager loop's (tests/test_gpu_graphs.py).

Data parallel (an initialised process group with world > 1): the trainer is built WITHOUT the
DDP wrapper (``SegmentTrainer(..., ddp=False)``) -- DDP's reducer hangs its hooks on the
parameters' gradient accumulators, which would then run inside the capture -- and
GraphedSegments does DDP's two jobs itself: at construction it broadcasts rank 0's parameters
(DDP's start-up broadcast), and ``step`` all-reduces the gradients after each replay (one flat
fp32 all-reduce of every gradient, divided by the world size as DDP's default hook does) before
the clip + Adam.  The all-reduce no longer overlaps the backward (DDP's buckets do); in exchange
the host issues ~0.2 ms per segment instead of ~2.8 ms.  The backend is the process group's
(RCCL on the GPUs; gloo in the one-GPU two-rank test, tests/test_gpu_ddp.py, bitwise equal to
eager DDP).

Restrictions, all checked: ``accumulation_steps == 1`` (every segment steps),
HIP Adam (optim.hip_adam_eligible), no per-launch timing events during capture
(ops.LAUNCH_EVENTS is None), no ``save_every_n_updates`` (periodic checkpoints are the
caller's: ``step`` replays and steps only).  The segments' tensors are the graphs' inputs:
overwrite them in place (``copy_``) to feed new data of the same shapes.  After ``step`` the
parameters' ``.grad`` are None again, as after the eager loop's ``zero_grad``.
"""
import gc
from typing import List, Optional

import torch

from . import ops
from .optim import hip_adam_eligible


class GraphedSegments:
    def __init__(self, trainer, segments: List[dict]):
        if trainer.ddp:
            raise ValueError("GraphedSegments: build the trainer with ddp=False; under a process "
                             "group of world > 1 the graphs broadcast and all-reduce themselves "
                             "(DDP's reducer hooks would run inside the capture)")
        if trainer.accumulation_steps != 1:
            raise ValueError("GraphedSegments: accumulation_steps must be 1")
        if not hip_adam_eligible(trainer.optimizer):
            raise ValueError("GraphedSegments: needs the HIP clip + Adam path "
                             "(optim.hip_adam_eligible)")
        if not segments or not all(s["feats"].is_cuda for s in segments):
            raise ValueError("GraphedSegments: segments must be device tensors")
        if trainer.save_every_n_updates:
            raise ValueError("GraphedSegments: periodic checkpoints (save_every_n_updates) are "
                             "the caller's in replay mode; build the trainer without them")
        self.trainer = trainer
        self.segments = segments
        self.params = [p for g in trainer.optimizer.param_groups for p in g["params"]
                       if p.requires_grad]
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.losses: List[torch.Tensor] = []
        self.grads: List[List[Optional[torch.Tensor]]] = []
        self.pos = 0
        import torch.distributed as dist
        self.ddp = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self._flat = None    # (data parallel) the flat all-reduce buffer, per-parameter views
        self._views = None
        if self.ddp:   # DDP's start-up broadcast: every rank starts from rank 0's weights
            with torch.no_grad():
                for p in self.params:
                    dist.broadcast(p.data, 0)
            ops.invalidate_weight_images()

    def _run(self, i, state):
        s = self.segments[i]
        return self.trainer.forward_backward(s["feats"], s["masks"], s["tokens"], s["in_lens"],
                                             s["tgt_lens"], state)

    def _allreduce(self, grads):
        """(DDP) this rank's gradients -> their mean over the ranks, as per-parameter views of
        one flat fp32 buffer: two copies and ONE all-reduce.  Returns the views."""
        import torch.distributed as dist
        if self._flat is None:
            n = sum(p.numel() for p in self.params)
            self._flat = torch.empty(n, dtype=torch.float32, device=self.params[0].device)
            self._views, off = [], 0
            for p in self.params:
                self._views.append(self._flat[off:off + p.numel()].view_as(p))
                off += p.numel()
        present = [(v, g) for v, g in zip(self._views, grads) if g is not None]
        if len(present) != len(self._views):
            self._flat.zero_()   # (a parameter without a gradient this segment: zeros, as DDP)
        if present:
            torch._foreach_copy_([v for v, _ in present], [g for _, g in present])
        dist.all_reduce(self._flat)
        self._flat.div_(dist.get_world_size())
        return self._views

    def capture(self, warmup: int = 1):
        """Warm every segment position up on a side stream (lazy library state: the capture
        stream's BLAS handle and workspace), then capture one graph per position."""
        if ops.LAUNCH_EVENTS is not None:
            raise RuntimeError("GraphedSegments.capture: per-launch timing events are on")
        dev = self.segments[0]["feats"].device
        # the eager loop's carried state still references its last autograd graph, whose
        # AccumulateGrad nodes belong to the eager stream: drop it (with them) before capturing
        self.trainer.encoder_state = None
        for p in self.params:
            p.grad = None
        gc.collect()
        torch.cuda.synchronize(dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                state = None
                for i in range(len(self.segments)):
                    _, state = self._run(i, state)
                    for p in self.params:
                        p.grad = None
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        state = None
        self.graphs, self.losses, self.grads = [], [], []   # (a second capture replaces the first)
        for i in range(len(self.segments)):
            ops.invalidate_weight_images()   # this graph builds (at replay) the images it reads
            for p in self.params:
                p.grad = None
            g = torch.cuda.CUDAGraph()
            # one memory pool for every position: replays run in capture order and what must
            # outlive a replay (state, gradients, loss) stays referenced, so position i + 1's
            # activations reuse position i's instead of holding one copy per position
            pool = self.graphs[0].pool() if self.graphs else None
            with torch.cuda.graph(g, pool=pool):
                loss, state = self._run(i, state)
            self.graphs.append(g)
            self.losses.append(loss)
            self.grads.append([p.grad for p in self.params])
        for p in self.params:
            p.grad = None
        ops.invalidate_weight_images()   # (the cache holds graph memory not yet written)
        self.pos = 0
        return self

    def begin_batch(self):
        """New server batch: the next replay is position 0 (no input state)."""
        self.pos = 0

    def step(self):
        """Replay the next segment position, then clip + Adam on its gradients.  Returns the
        (graph-owned) loss tensor of that segment."""
        if not self.graphs:
            raise RuntimeError("GraphedSegments.step before capture()")
        i = self.pos
        self.graphs[i].replay()
        grads = self._allreduce(self.grads[i]) if self.ddp else self.grads[i]
        for p, g in zip(self.params, grads):
            p.grad = g
        self.trainer._clip_and_step()
        for p in self.params:   # as the eager loop's zero_grad(set_to_none=True): no caller
            p.grad = None       # backward may accumulate into graph-owned gradient memory
        self.trainer.global_step += 1
        self.pos = (i + 1) % len(self.graphs)
        return self.losses[i]
