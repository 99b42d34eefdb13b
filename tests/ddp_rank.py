"""One rank of the two-rank training runs on a single GPU (tests/test_gpu_ddp.py::test_*_two_ranks_*).

    python tests/ddp_rank.py RANK WORLD PORT ACCUMULATION OUT.pt [WORKLOAD [OPTIM [MODE]]]

WORKLOAD (default c3), each on a 4-sequence batch, 4 segments with the encoder state carried,
bf16 autocast, 8 MB buckets:
  c3  LucyRNN 6 x 512 + CTC, V = 1024, T = 1500, U <= 150 (config C3's model and step);
  c4  xLSTM 2 blocks x 768 (mLSTM, 4 heads, the reference's float16 cell) + CTC, T = 1536: the
      encoder state is the xLSTM's dict of per-block tuples (/root/reference/model.py:17-18);
  c5  LucyRNN 6 x 512 + RNN-T with the fused joiner, U = 150: encoder AND joiner under DDP, one
      optimizer over both (/root/reference/model.py:73-145, train.py:144-146).
OPTIM: adam (the reference's optim.Adam(lr 3e-4), stepped by the HIP clip + Adam) or sgd
(torch.optim.SGD(lr 1e-3) after clip_grad_norm_: no sign normalisation, so reduction-order noise
stays proportional to itself through the later steps).
MODE: eager (SegmentTrainer.train_segment, DDP's bucket hooks), graph (graphs.GraphedSegments:
each segment's forward + backward captured once and replayed, the gradients all-reduced after
the replay; no DDP wrapper; adam, accumulation 1) or split (WORLD 1: the two ranks' halves as two
micro-batches of one process with their own carried states, gradients summed and halved).

WORLD = 2 ranks train rows [2 r, 2 r + 2) each under DistributedDataParallel over a "gloo" group
(both ranks on cuda:0 -- RCCL refuses two ranks on one device; gloo all-reduces the CUDA
gradients through host memory); WORLD = 1 trains all four rows in one process without DDP.
Rank r initialises its modules with seed 11 + 1000 r and (LucyRNN) runs one no-grad forward
BEFORE the DDP wrap, so its cached bf16 weight images hold its OWN weights: DDP's start-up
broadcast of rank 0's parameters must reach them.  After every segment rank 0 gathers rank 1's
flattened parameters and records whether they are bitwise its own.  The gradients the first
optimizer step sees (after DDP's all-reduce, before the clip + step) are captured.  OUT.pt holds
the losses, those flags, and (rank 0 / the single process) the captured gradients and the
parameters before the first and after the last step."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

V, BFULL, SEGS = 1024, 4, 4


def batch(seg, T, U):
    """Segment `seg` of the full 4-row batch, identical on every rank (each takes its rows)."""
    g = torch.Generator().manual_seed(7 + seg)
    feats = torch.randn(BFULL, T, 80, generator=g)
    tok = torch.randint(1, V, (BFULL, U), generator=g)
    tl = [U, 97, 131, 64]
    for b in range(BFULL):
        tok[b, tl[b]:] = 0
    return feats, tok, tl


def build(workload, dev):
    """(model, joiner or None, criterion, mode, T, U)"""
    from statecatcher_amd.model import (ASRModel, CTCLoss, RNNTLoss, RNNTPredictorJoiner,
                                        build_lucyrnn_config, build_xlstm_config)
    if workload == "c4":
        cfg = build_xlstm_config(80, V, num_heads=4, num_blocks=2, embedding_dim=768)
        model = ASRModel(None, cfg, vocab_size=V, feat_dim=80, proj_dim=-1).to(dev)
        return model, None, CTCLoss(blank=0, zero_infinity=True), "ctc", 1536, 150
    model = ASRModel(None, build_lucyrnn_config(80, 512, 6, V), vocab_size=V, feat_dim=80,
                     proj_dim=-1).to(dev)
    with torch.no_grad():
        model.encoder.output_proj.weight.normal_(0, 0.02)
    if workload == "c5":
        joiner = RNNTPredictorJoiner(V, 64, 64, V).to(dev)
        return model, joiner, RNNTLoss(blank=0, fused_joint=True), "rnnt", 1500, 150
    return model, None, CTCLoss(blank=0, zero_infinity=True), "ctc", 1500, 150


def main():
    rank, world, port, acc, out = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]),
                                   int(sys.argv[4]), sys.argv[5])
    workload = sys.argv[6] if len(sys.argv) > 6 else "c3"
    optim = sys.argv[7] if len(sys.argv) > 7 else "adam"
    mode_run = sys.argv[8] if len(sys.argv) > 8 else "eager"
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    if world > 1:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
    import statecatcher_amd.train as train_mod
    from statecatcher_amd.train import SegmentTrainer
    first_grads = []
    orig_step = train_mod.clip_and_adam_step

    def capture(opt, params, max_norm):   # the all-reduced gradients of the first update
        if not first_grads:
            first_grads.extend(p.grad.detach().float().cpu().clone() for p in all_params)
        return orig_step(opt, params, max_norm)
    train_mod.clip_and_adam_step = capture
    torch.manual_seed(11 + 1000 * rank)
    model, joiner, crit, mode, T, U = build(workload, dev)
    if workload != "c4":
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):   # OWN weight images
            model(torch.randn(1, 64, 80, device=dev), torch.ones(1, 64, dtype=torch.bool, device=dev))
    all_params = list(model.parameters()) + ([] if joiner is None else list(joiner.parameters()))
    if optim == "sgd":
        opt = torch.optim.SGD(all_params, lr=1e-3)
        orig_opt_step = opt.step

        def sgd_step(*a, **k):   # the SGD path's first update: capture its gradients too
            if not first_grads:
                first_grads.extend(p.grad.detach().float().cpu().clone() for p in all_params)
            return orig_opt_step(*a, **k)
        opt.step = sgd_step
    else:
        opt = torch.optim.Adam(all_params, lr=3e-4)
    kw = dict(mode="rnnt", joiner=joiner) if mode == "rnnt" else {}
    # graph mode: no DDP wrapper (its reducer's hooks sit on the parameters' gradient
    # accumulators and would run inside the capture); GraphedSegments broadcasts rank 0's
    # weights and all-reduces the gradients itself
    ddp = world > 1 and mode_run != "graph"
    tr = SegmentTrainer(model, crit, opt, amp_dtype=torch.bfloat16, max_grad_norm=50.0,
                        bucket_cap_mb=8.0, accumulation_steps=acc, ddp=ddp, **kw)
    if ddp:
        assert isinstance(tr.net, torch.nn.parallel.DistributedDataParallel)
        assert tr.net.bucket_bytes_cap == 8 * 1024 * 1024
        if joiner is not None:
            assert isinstance(tr.joiner_net, torch.nn.parallel.DistributedDataParallel)
    # split (WORLD 1): the two ranks' halves as two micro-batches of ONE process, each with its
    # own carried state, gradients summed and halved before the clip + step -- the arithmetic of a
    # two-rank DDP step done without DDP (tests/test_gpu_ddp.py: bitwise equal to it)
    halves = 2 if mode_run == "split" else 1
    B = BFULL // (world * halves)

    def rows_of(r):
        return slice(r * B, (r + 1) * B)
    segs = []   # this rank's rows of the 4 segments, device-resident (as bench.py feeds them)
    for seg in range(SEGS):
        feats, tok, tl = batch(seg, T, U)
        per = []
        for hh in range(halves):
            rows = rows_of(rank * halves + hh)
            per.append(dict(feats=feats[rows].to(dev),
                            masks=torch.ones(B, T, dtype=torch.bool, device=dev),
                            tokens=tok[rows].to(dev),
                            in_lens=torch.full((B,), T, dtype=torch.int64, device=dev),
                            tgt_lens=torch.tensor(tl[rows], dtype=torch.int64, device=dev)))
        segs.append(per)
    graphed = None
    if mode_run == "graph":
        from statecatcher_amd.graphs import GraphedSegments
        graphed = GraphedSegments(tr, [sg[0] for sg in segs])   # (broadcasts rank 0's weights)
    init = [p.detach().cpu().clone() for p in all_params]   # (rank 0's, broadcast)
    if graphed is not None:
        graphed.capture()
        graphed.begin_batch()
    tr.begin_batch()
    losses, equal = [], []
    states = [None] * halves
    for seg in range(SEGS):
        if graphed is not None:
            loss = float(graphed.step().detach())
        elif mode_run == "split":
            assert world == 1 and acc == 1
            loss = []
            for hh in range(halves):
                sg = segs[seg][hh]
                lh, states[hh] = tr.forward_backward(sg["feats"], sg["masks"], sg["tokens"],
                                                     sg["in_lens"], sg["tgt_lens"], states[hh])
                loss.append(float(lh.detach()))
            for p in all_params:
                if p.grad is not None:
                    p.grad.div_(halves)
            tr._clip_and_step()
            tr.optimizer.zero_grad(set_to_none=True)
        else:
            sg = segs[seg][0]
            loss = float(tr.train_segment(sg["feats"], sg["masks"], sg["tokens"], sg["in_lens"],
                                          sg["tgt_lens"]).detach())
        losses.append(loss)
        if world > 1:
            flat = torch.cat([p.detach().reshape(-1) for p in all_params])
            got = [torch.empty_like(flat) for _ in range(world)]
            dist.all_gather(got, flat)
            equal.append(all(torch.equal(got[0], x) for x in got[1:]))
    torch.cuda.synchronize()
    if workload == "c4" and graphed is None and mode_run != "split":
        st = tr.encoder_state   # the carried state is the xLSTM's dict of per-block tuples
        assert isinstance(st, dict) and st, type(st)
    res = {"losses": losses, "ranks_bitwise_equal": equal}
    if rank == 0:
        res["init"] = init
        res["params"] = [p.detach().cpu() for p in all_params]
        res["grads"] = first_grads
    torch.save(res, out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
