"""RCCL readiness on the leased GPU: SegmentTrainer wrapped in DistributedDataParallel over a
1-rank "nccl" (= RCCL) process group, with the HIP ops and the HIP clip + Adam underneath.

The reference trains single-process (/root/reference/train.py:85-89, :460-581); data-parallel
training is this build's addition.  A 1-GPU lease cannot run a multi-rank
collective, so this runs the real RCCL communicator at world size 1: DDP's bucket hooks fire over
LucyCellFn's fused bias gradient, gradient_as_bucket_view buckets meet optim.clip_and_adam_step,
and every bucket is all-reduced through RCCL.  The 2-rank sharding semantics are covered on the CPU
by tests/test_train_ddp.py (gloo).  Parameters after 2 segments (state carried) must be BITWISE
equal to the same training without DDP -- on a small model, and on config C3's (6 x 512, V 1024,
T 1500, 8 MB buckets, 4 carried segments, accumulation 1 and 2).
"""
import os

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def sc():
    import statecatcher_amd as s
    return s


@pytest.fixture(scope="module")
def rccl_group():
    import socket
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=DEV)
    assert dist.get_backend() == "nccl"
    yield
    dist.destroy_process_group()


def _build(mode, seed=0):
    from statecatcher_amd.model import (ASRModel, CTCLoss, RNNTLoss, RNNTPredictorJoiner,
                                        build_lucyrnn_config)
    torch.manual_seed(seed)
    V = 256
    model = ASRModel(None, build_lucyrnn_config(80, 256, 3, V), vocab_size=V, feat_dim=80,
                     proj_dim=-1).to(DEV)
    with torch.no_grad():
        model.encoder.output_proj.weight.normal_(0, 0.02)
    if mode == "rnnt":
        joiner = RNNTPredictorJoiner(V, 64, 64, V).to(DEV)
        return model, joiner, RNNTLoss(blank=0), list(model.parameters()) + list(joiner.parameters())
    return model, None, CTCLoss(blank=0, zero_infinity=True), list(model.parameters())


def _train(mode, ddp):
    from statecatcher_amd.train import SegmentTrainer
    model, joiner, crit, params = _build(mode)
    opt = torch.optim.Adam(params, lr=3e-4)
    kw = dict(mode=mode, joiner=joiner) if mode == "rnnt" else {}
    tr = SegmentTrainer(model, crit, opt, amp_dtype=torch.bfloat16, max_grad_norm=50.0,
                        bucket_cap_mb=1.0, ddp=ddp, **kw)
    if ddp:
        assert isinstance(tr.net, torch.nn.parallel.DistributedDataParallel)
    g = torch.Generator().manual_seed(5)
    B, T = 4, 300
    tr.begin_batch()
    losses = []
    for _ in range(2):   # two segments, encoder state carried (detached) between them
        feats = torch.randn(B, T, 80, generator=g).to(DEV)
        tok = torch.randint(1, 256, (B, 20), generator=g).to(DEV)
        loss = tr.train_segment(feats, torch.ones(B, T, dtype=torch.bool, device=DEV), tok,
                                [T] * B, [20, 17, 12, 20])
        losses.append(float(loss.detach()))
    torch.cuda.synchronize()
    return losses, [p.detach().clone() for p in params]


@pytest.mark.parametrize("mode", ["ctc", "rnnt"])
def test_ddp_over_rccl_equals_single_process(rccl_group, mode):
    l_ref, p_ref = _train(mode, ddp=False)
    l_ddp, p_ddp = _train(mode, ddp=True)
    print(f"{mode}: losses {l_ref} (plain) {l_ddp} (DDP over RCCL)")
    assert l_ref == l_ddp
    for a, b in zip(p_ref, p_ddp):
        assert torch.equal(a, b)
    # the parameters moved: the all-reduced gradients reached the HIP Adam
    _, _, _, p0 = _build(mode)
    assert any(not torch.equal(a, b) for a, b in zip(p_ref, p0))


@pytest.mark.parametrize("accumulation", [1, 2])
def test_c3_model_ddp_over_rccl_equals_single_process(rccl_group, accumulation):
    """Config C3's model and step as bench.py runs it: LucyRNN 6 x 512 + CTC, V = 1024, T = 1500,
    bf16 autocast, the bench's 8 MB buckets (the 40 MB of gradients in 5+ buckets, each layer's
    all-reduce overlapping the backward below it), 4 segments with the encoder state carried, and
    gradient accumulation over 1 and 2 segments (no_sync on the accumulating ones); B = 2 per rank.
    DDP over the RCCL communicator must leave every parameter bitwise where plain training does."""
    from statecatcher_amd.model import ASRModel, CTCLoss, build_lucyrnn_config
    from statecatcher_amd.train import SegmentTrainer
    V, B, T, U = 1024, 2, 1500, 150

    def run(ddp):
        torch.manual_seed(11)
        model = ASRModel(None, build_lucyrnn_config(80, 512, 6, V), vocab_size=V, feat_dim=80,
                         proj_dim=-1).to(DEV)
        with torch.no_grad():
            model.encoder.output_proj.weight.normal_(0, 0.02)
        params = list(model.parameters())
        opt = torch.optim.Adam(params, lr=3e-4)
        tr = SegmentTrainer(model, CTCLoss(blank=0, zero_infinity=True), opt,
                            amp_dtype=torch.bfloat16, max_grad_norm=50.0, bucket_cap_mb=8.0,
                            accumulation_steps=accumulation, ddp=ddp)
        if ddp:   # the bench's bucket cap: 40 MB of gradients in 5+ all-reduces
            assert tr.net.bucket_bytes_cap == 8 * 1024 * 1024
        g = torch.Generator().manual_seed(7)
        tr.begin_batch()
        losses = []
        for _ in range(4):
            feats = torch.randn(B, T, 80, generator=g).to(DEV)
            tok = torch.randint(1, V, (B, U), generator=g).to(DEV)
            loss = tr.train_segment(feats, torch.ones(B, T, dtype=torch.bool, device=DEV), tok,
                                    [T] * B, [U, 97])
            losses.append(float(loss.detach()))
        torch.cuda.synchronize()
        state = [t.detach().clone() for t in tr.encoder_state[0][0] + tr.encoder_state[1][0]]
        return losses, [p.detach().clone() for p in params], state

    l_ref, p_ref, s_ref = run(False)
    l_ddp, p_ddp, s_ddp = run(True)
    print(f"C3 acc={accumulation}: losses {l_ref} (plain) {l_ddp} (DDP over RCCL)")
    assert l_ref == l_ddp
    assert all(torch.equal(a, b) for a, b in zip(p_ref, p_ddp))
    assert all(torch.equal(a, b) for a, b in zip(s_ref, s_ddp))
    assert all(torch.isfinite(torch.tensor(l_ref)))


def _run_ranks(world, acc, tmp_path, workload="c3", optim="adam", mode="eager"):
    """tests/ddp_rank.py as `world` fresh processes (none forked from this HIP-initialised one),
    with a common deadline; returns each rank's saved results."""
    import socket
    import subprocess
    import sys
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = [str(tmp_path / f"{workload}_{optim}_{mode}_w{world}_a{acc}_r{r}.pt")
            for r in range(world)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(root, "tests", "ddp_rank.py"), str(r),
                               str(world), str(port), str(acc), outs[r], workload, optim, mode],
                              cwd=root, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True)
             for r in range(world)]
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=150)[0])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return [torch.load(o, weights_only=True) for o in outs]


def _rel(a, b):
    return float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))


def _two_rank_case(workload, optim, acc, tmp_path):
    """Two ranks (B = 2 each) against one process on the full B = 4 batch; returns the measured
    errors after checking what holds exactly: ranks bitwise equal after every segment."""
    single = _run_ranks(1, acc, tmp_path, workload, optim)[0]
    r0, r1 = _run_ranks(2, acc, tmp_path, workload, optim)
    assert r0["ranks_bitwise_equal"] == [True] * 4 and r1["ranks_bitwise_equal"] == [True] * 4
    assert all(torch.equal(a, b) for a, b in zip(r0["init"], single["init"]))
    lr = {"adam": 3e-4, "sgd": 1e-3}[optim]
    e = {"loss": [abs((a + b) / 2 - s) / abs(s) for a, b, s in
                  zip(r0["losses"], r1["losses"], single["losses"])],
         "grad": [_rel(a, b) for a, b in zip(r0["grads"], single["grads"])],
         # the parameters after the last step, and the update they made from the common start
         "param": [_rel(a, b) for a, b in zip(r0["params"], single["params"])],
         "update": [_rel(a - i, b - i) for a, b, i in
                    zip(r0["params"], single["params"], single["init"])],
         # the largest element-wise parameter difference, in units of lr x steps taken
         "flip": max(float((a.double() - b.double()).abs().max()) for a, b in
                     zip(r0["params"], single["params"])) / (lr * (4 // acc)),
         "numel": [a.numel() for a in r0["params"]],
         # the whole first-update gradient as one vector (small tensors whose gradient nearly
         # cancels weigh by their size)
         "grad_all": _rel(torch.cat([a.reshape(-1) for a in r0["grads"]]),
                          torch.cat([b.reshape(-1) for b in single["grads"]]))}
    assert len(e["grad"]) == len(r0["params"]) and all(map(lambda x: x == x, e["update"]))
    print(f"{workload} {optim} acc={acc}: losses {r0['losses']} / {r1['losses']} vs "
          f"{single['losses']}; loss rel {['%.1e' % x for x in e['loss']]}; first-update gradient "
          f"rel max {max(e['grad']):.2e} ({len(e['grad'])} tensors); final param rel max "
          f"{max(e['param']):.2e}; update rel max {max(e['update']):.2e} median "
          f"{sorted(e['update'])[len(e['update']) // 2]:.2e}; largest element difference "
          f"{e['flip']:.2f} lr-steps")
    print("  per tensor (numel, first-update gradient rel, param rel, update rel):",
          [(n, f"{g:.1e}", f"{p:.1e}", f"{u:.1e}")
           for n, g, p, u in zip(e["numel"], e["grad"], e["param"], e["update"])])
    return e


@pytest.mark.parametrize("accumulation", [1, 2])
def test_c3_two_ranks_on_one_gpu_equal_one_process_on_the_full_batch(accumulation, tmp_path):
    """Config C3's sharding with the real HIP model at world size 2 (verdict r4 item 1, r5 item 2):
    two rank processes on cuda:0 over a gloo group, B = 2 each (tests/ddp_rank.py), against one
    process training the same B = 4 batch with the reference's Adam.  Rank 1 starts from DIFFERENT
    weights and has built its bf16 weight images from them before the DDP wrap, so DDP's start-up
    broadcast must reach the version-keyed image cache.  Done when:
      * both ranks' parameters are bitwise equal after every segment;
      * until the first optimizer step (identical weights), the mean of the per-rank losses (each
        the mean of its sequences' nll / U) is the full-batch loss (CTC 'mean' over equal shards);
      * the gradients that step applies -- all-reduced over the ranks, with rank 1's shard
        computed from the broadcast weights -- are the full-batch gradients (relative Frobenius
        per tensor, <= 1e-4; the runs differ only in reduction order: GEMM row counts, split-L
        slabs, the all-reduce);
      * every later segment's loss stays within north_star's 1e-3 of the full-batch run's;
      * the final parameters part only the way Adam's sign normalisation allows.  Adam's first
        update is exactly -lr sign(g) per element (m / sqrt(v) = g / |g| after bias correction),
        so an element whose gradient is at the reduction-order noise level moves +-lr whichever
        way the noise tips it: measured, the first update's gradients agree to 1.6e-7 in norm, yet
        the runs' total updates differ by 0.1-0.3 relative on every tensor (a few % of the
        elements flipped), the largest element difference is 0.79 lr-steps, and the parameters
        themselves (weight matrices) 2e-5 .. 5.6e-3 relative.  Pinned: no element more than 2 lr
        per step apart (the mechanism's bound), every weight matrix (>= 64 K elements) within
        1e-2.  test_c3_two_ranks_sgd_stay_equal_through_every_step pins the multi-step equality
        itself, without the sign normalisation.
    Accumulation 1 and 2 (no_sync on the accumulating segments)."""
    e = _two_rank_case("c3", "adam", accumulation, tmp_path)
    for x in e["loss"][:accumulation]:   # identical weights: reduction order only
        assert x <= 1e-5, e["loss"]
    # measured 3e-7 (acc 1) and 1.1e-5 (acc 2: the second segment's state was carried from the
    # first segment's split-batch scans, so two steps of reduction-order noise); north_star's
    # 1e-3 is the bar, 1e-4 leaves 10x of it for the reduction order alone
    assert max(e["grad"]) <= 1e-4, e["grad"]
    _adam_bounds(e)


def _adam_bounds(e):
    assert max(e["loss"]) <= 1e-3, e["loss"]
    assert e["flip"] <= 2.0, e["flip"]
    big = [p for p, n in zip(e["param"], e["numel"]) if n >= 65536]
    assert big and max(big) <= 1e-2, big


def test_c3_two_ranks_sgd_stay_equal_through_every_step(tmp_path):
    """The multi-step leg without Adam's sign normalisation (verdict r5 item 2): with
    clip_grad_norm_ + torch.optim.SGD the reduction-order noise of each step stays proportional
    to itself, so DDP training must STAY equal to single-process training through all 4 steps:
    every loss within 1e-4 and every tensor's total update (final - initial parameters) within
    1e-4 relative."""
    e = _two_rank_case("c3", "sgd", 1, tmp_path)
    assert max(e["grad"]) <= 1e-4, e["grad"]
    assert max(e["loss"]) <= 1e-4, e["loss"]
    assert max(e["update"]) <= 1e-4, e["update"]


@pytest.mark.parametrize("workload", ["c4", "c5"])
def test_c4_c5_two_ranks_on_one_gpu_equal_one_process_on_the_full_batch(workload, tmp_path):
    """The other north-star workloads at world size 2 on the HIP kernels (verdict r5 item 2):
      * c4: the xLSTM encoder (2 blocks x 768, T = 1536, mLSTM on the float16 cell), whose
        carried state is a dict of per-block tuples (/root/reference/model.py:17-18);
      * c5: LucyRNN 6 x 512 + RNN-T with the fused joiner (U = 150), encoder and joiner both
        DDP modules with their own buckets and one optimizer (model.py:73-145).
    Against one process on the full B = 4 batch the first loss is equal to 1e-5, but unlike C3
    (whose GEMM shapes the shipped TunableOp table pins to one kernel for any row count) the
    xLSTM projections and the joiner's enc / pred projections run library GEMMs whose kernel
    the library picks by the row count (B = 2 vs 4): their bf16 outputs differ by an ulp here and
    there, so the first update's gradients agree only at bf16 level (measured 4e-3 (c4) / 2.3e-3
    (c5) on the largest tensors, 0.57 on a 4-element gate bias whose gradient nearly cancels).
    Pinned here: the first loss to 1e-5, the whole first-update gradient to 1e-2, every loss to
    5e-3, no parameter element more than 2 lr per step apart (Adam's sign-flip bound).  That
    DDP itself adds nothing is pinned bitwise by
    test_two_ranks_bitwise_equal_to_split_batch_single_process."""
    e = _two_rank_case(workload, "adam", 1, tmp_path)
    assert e["loss"][0] <= 1e-5, e["loss"]
    assert e["grad_all"] <= 1e-2, e["grad_all"]
    assert max(e["loss"]) <= 5e-3, e["loss"]
    assert e["flip"] <= 2.0, e["flip"]


@pytest.mark.parametrize("workload", ["c3", "c4", "c5"])
def test_two_ranks_bitwise_equal_to_split_batch_single_process(workload, tmp_path):
    """DDP adds nothing to the arithmetic: two rank processes (B = 2 each, DDP over gloo, 4
    segments with carried state, the HIP clip + Adam) against ONE process that runs the same two
    halves as two micro-batches with their own carried states, sums their gradients, halves them
    and steps (tests/ddp_rank.py mode split): the same kernels at the same row counts, and a
    two-rank mean is one fp32 add and an exact halving however it is bucketed, so every loss of
    every half and every parameter after the 4 updates must be BITWISE equal -- for the LucyRNN
    + CTC step (c3), the xLSTM encoder with its dict state (c4) and the RNN-T encoder + joiner
    as two DDP modules (c5)."""
    split = _run_ranks(1, 1, tmp_path, workload, "adam", "split")[0]
    r0, r1 = _run_ranks(2, 1, tmp_path, workload, "adam", "eager")
    assert r0["ranks_bitwise_equal"] == [True] * 4
    print(f"{workload}: split halves {split['losses']}; ranks {r0['losses']} / {r1['losses']}")
    assert [l[0] for l in split["losses"]] == r0["losses"]
    assert [l[1] for l in split["losses"]] == r1["losses"]
    assert all(torch.equal(a, b) for a, b in zip(r0["params"], split["params"]))
    assert any(not torch.equal(a, b) for a, b in zip(r0["params"], r0["init"]))


@pytest.mark.parametrize("workload", ["c3", "c4", "c5"])
def test_graph_replay_ddp_two_ranks_bitwise_equal_to_eager_ddp(workload, tmp_path):
    """Data-parallel training under HIP-graph replay (verdict r5 item 8): two rank processes on
    cuda:0 over gloo, each capturing its 4 segment positions (graphs.GraphedSegments on a trainer
    without the DDP wrapper: rank 0's weights broadcast at construction, the bare forward +
    backward in the graph, one flat all-reduce of the gradients after each replay, then the HIP
    clip + Adam), against the same two ranks training eagerly under DDP's bucket hooks.  The
    per-rank gradients are the same kernels' and a two-rank mean is one fp32 add and an exact
    halving whichever way it is bucketed, so losses and parameters must be BITWISE equal after
    all 4 segments, and the ranks bitwise equal to each other throughout.  c5: the joiner's
    gradients ride in the same flat all-reduce."""
    eager = _run_ranks(2, 1, tmp_path, workload, "adam", "eager")
    graph = _run_ranks(2, 1, tmp_path, workload, "adam", "graph")
    for r in graph:
        assert r["ranks_bitwise_equal"] == [True] * 4
    print(f"{workload}: eager DDP losses {eager[0]['losses']} / {eager[1]['losses']}, graph "
          f"{graph[0]['losses']} / {graph[1]['losses']}")
    assert graph[0]["losses"] == eager[0]["losses"] and graph[1]["losses"] == eager[1]["losses"]
    assert all(torch.equal(a, b) for a, b in zip(graph[0]["params"], eager[0]["params"]))
    # and training moved the weights
    assert any(not torch.equal(a, b) for a, b in zip(graph[0]["params"], graph[0]["init"]))


def test_rccl_allreduce_of_a_gradient_sized_buffer(rccl_group):
    """The collective DDP issues, on its own: an fp32 all-reduce of the C2 gradient volume
    (10.0 M parameters) through RCCL at world size 1 is the identity."""
    x = torch.randn(10_013_696, device=DEV)
    y = x.clone()
    dist.all_reduce(y)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
