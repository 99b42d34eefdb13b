"""graphs.GraphedSegments: the segment loop's forward + backward replayed as HIP graphs must train
exactly as the eager SegmentTrainer does (/root/reference/train.py:460-581: state reset per server
batch, state carried between segments, clip + Adam after every segment).

Two copies of one model from one seed, the same fixed device-resident segments: the eager loop
(train_segment, begin_batch every n segments) against the graphed one (capture once, replay).
The same kernels run in the same order on the same data, so the per-segment losses and every
parameter after two server batches (2 x n optimizer steps) must be BITWISE equal -- which also
proves each graph rebuilt the bf16 weight images after every Adam step (a stale image would
change the second segment's loss) and that graph i read graph i - 1's output state."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _segments(n, B, T, V, U, seed):
    g = torch.Generator().manual_seed(seed)
    segs = []
    for _ in range(n):
        lens = torch.randint(U // 2, U + 1, (B,), generator=g)
        tok = torch.randint(1, V, (B, U), generator=g)
        for b in range(B):
            tok[b, lens[b]:] = 0
        segs.append(dict(feats=torch.randn(B, T, 80, generator=g).to(DEV),
                         masks=torch.ones(B, T, dtype=torch.bool, device=DEV),
                         tokens=tok.to(DEV), in_lens=torch.full((B,), T, device=DEV),
                         tgt_lens=lens.to(DEV)))
    return segs


def _trainer(mode, layers, hidden, V, seed=3):
    from statecatcher_amd.model import (ASRModel, CTCLoss, RNNTLoss, RNNTPredictorJoiner,
                                        build_lucyrnn_config, build_xlstm_config)
    from statecatcher_amd.train import SegmentTrainer
    torch.manual_seed(seed)
    if mode == "xlstm":   # C4's encoder family: layers = blocks, hidden = embedding_dim
        cfg = build_xlstm_config(80, V, num_heads=2, num_blocks=layers, embedding_dim=hidden)
        model = ASRModel(None, cfg, vocab_size=V, feat_dim=80, proj_dim=-1).to(DEV)
    else:
        model = ASRModel(None, build_lucyrnn_config(80, hidden, layers, V), vocab_size=V,
                         feat_dim=80, proj_dim=-1).to(DEV)
        with torch.no_grad():
            model.encoder.output_proj.weight.normal_(0, 0.02)
    params = list(model.parameters())
    kw = {}
    crit = CTCLoss(blank=0, zero_infinity=True)
    if mode == "rnnt":
        joiner = RNNTPredictorJoiner(V, 64, 64, V).to(DEV)
        params += list(joiner.parameters())
        kw = dict(mode="rnnt", joiner=joiner)
        crit = RNNTLoss(blank=0)
    opt = torch.optim.Adam(params, lr=3e-4)
    tr = SegmentTrainer(model, crit, opt, amp_dtype=torch.bfloat16, max_grad_norm=50.0, **kw)
    return tr, params


@pytest.mark.parametrize("mode,layers,hidden,V,B,T,U", [
    ("ctc", 3, 256, 256, 4, 300, 20),
    ("ctc", 6, 512, 1024, 2, 1500, 150),   # config C2's model and segment length
    ("rnnt", 2, 256, 256, 2, 200, 12),
    ("xlstm", 2, 256, 256, 2, 256, 20),    # C4's encoder (mLSTM blocks) + CTC
])
def test_graphed_segments_train_bitwise_as_the_eager_loop(mode, layers, hidden, V, B, T, U):
    from statecatcher_amd.graphs import GraphedSegments
    n = 3
    segs = _segments(n, B, T, V, U, seed=9)

    tr, p_eager = _trainer(mode, layers, hidden, V)
    l_eager = []
    for k in range(2 * n):
        if k % n == 0:
            tr.begin_batch()
        s = segs[k % n]
        l_eager.append(tr.train_segment(s["feats"], s["masks"], s["tokens"], s["in_lens"],
                                        s["tgt_lens"]).detach().clone())
    torch.cuda.synchronize()

    tr2, p_graph = _trainer(mode, layers, hidden, V)
    gs = GraphedSegments(tr2, segs).capture()
    # capture changed nothing: no optimizer step, the parameters are the initial ones
    _, p_init = _trainer(mode, layers, hidden, V)
    assert all(torch.equal(a, b) for a, b in zip(p_graph, p_init))
    l_graph = []
    for k in range(2 * n):
        if k % n == 0:
            gs.begin_batch()
        l_graph.append(gs.step().detach().clone())
    torch.cuda.synchronize()
    print(f"{mode} L{layers}x{hidden}: eager {[float(x) for x in l_eager]} "
          f"graphed {[float(x) for x in l_graph]}")
    assert all(torch.isfinite(x).all() for x in l_eager)
    assert all(torch.equal(a, b) for a, b in zip(l_eager, l_graph))
    assert all(torch.equal(a, b) for a, b in zip(p_eager, p_graph))
    # and training moved the weights
    assert any(not torch.equal(a, b) for a, b in zip(p_eager, p_init))


def test_capture_after_eager_steps_continues_the_eager_run():
    """bench.py's order: eager warmup steps on the trainer, then capture on the same trainer (its
    carried state still holding the last eager autograd graph), then replays -- which must
    continue exactly where the eager run would have gone."""
    from statecatcher_amd.graphs import GraphedSegments
    n = 2
    segs = _segments(n, 4, 300, 256, 20, seed=4)

    def eager_steps(tr, k0, k1):
        out = []
        for k in range(k0, k1):
            if k % n == 0:
                tr.begin_batch()
            s = segs[k % n]
            out.append(tr.train_segment(s["feats"], s["masks"], s["tokens"], s["in_lens"],
                                        s["tgt_lens"]).detach().clone())
        return out

    tr_a, p_a = _trainer("ctc", 3, 256, 256)
    la = eager_steps(tr_a, 0, 3 * n)
    tr_b, p_b = _trainer("ctc", 3, 256, 256)
    lb = eager_steps(tr_b, 0, n)
    gs = GraphedSegments(tr_b, segs).capture()
    for k in range(n, 3 * n):
        if k % n == 0:
            gs.begin_batch()
        lb.append(gs.step().detach().clone())
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(la, lb))
    assert all(torch.equal(a, b) for a, b in zip(p_a, p_b))


def test_bench_graph_mode_prints_its_line():
    """`bench.py --graph on` end to end at a small size (a child process: the bench owns its
    process): one JSON line with the replay named in `launch` and the kernel timings taken from
    the eager steps after the timed region."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "bench.py", "--graph", "on", "--steps", "4", "--warmup", "2",
                        "--batch", "2", "--seq", "300", "--segments", "2", "--cpu-baseline", "off"],
                       cwd=root, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["launch"].startswith("hip-graph") and "eager steps" in line["kernel_timing"]
    assert line["value"] > 0 and line["roofline"]["achieved"] > 0
    assert line["kernels"]["lucy_scan_bwd"]["launches"] > 0


def test_graphed_segments_refuse_what_they_cannot_capture():
    from statecatcher_amd import ops
    from statecatcher_amd.graphs import GraphedSegments
    from statecatcher_amd.train import SegmentTrainer
    tr, _ = _trainer("ctc", 1, 256, 256)
    segs = _segments(1, 2, 64, 256, 8, seed=1)
    acc = SegmentTrainer(tr.model, tr.criterion, tr.optimizer, accumulation_steps=2)
    with pytest.raises(ValueError):
        GraphedSegments(acc, segs)
    with pytest.raises(RuntimeError):
        GraphedSegments(tr, segs).step()
    ops.LAUNCH_EVENTS = []
    try:
        with pytest.raises(RuntimeError):
            GraphedSegments(tr, segs).capture()
    finally:
        ops.LAUNCH_EVENTS = None
