"""One rank of the two-rank C3 run on a single GPU (tests/test_gpu_ddp.py::test_c3_two_ranks_*).

    python tests/c3_rank.py RANK WORLD PORT ACCUMULATION OUT.pt

Config C3's model and step (LucyRNN 6 x 512 + CTC, V = 1024, T = 1500, bf16 autocast with the
split-precision output head, 8 MB buckets, 4 segments with the encoder state carried) on a
4-sequence batch: WORLD = 2 ranks train rows [2 r, 2 r + 2) each under DistributedDataParallel
over a "gloo" group (both ranks on cuda:0 -- RCCL refuses two ranks on one device; gloo
all-reduces the CUDA gradients through host memory), WORLD = 1 trains all four rows in one
process without DDP.

Rank r initialises its model with seed 11 + 1000 r and runs one no-grad forward BEFORE the DDP
wrap, so its cached bf16 weight images (ops.weight_images, keyed on the parameters' version
counters) hold its OWN weights: DDP's start-up broadcast of rank 0's parameters must reach them.
After every segment rank 0 gathers rank 1's flattened parameters and records whether they are
bitwise its own.  The gradients the first optimizer step sees (after DDP's all-reduce, before the
HIP clip + Adam) are captured.  OUT.pt holds the losses, those flags, the captured gradients and
the final parameters (rank 0 / the single process only)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

V, T, U, BFULL, SEGS = 1024, 1500, 150, 4, 4


def batch(seg):
    """Segment `seg` of the full 4-row batch, identical on every rank (each takes its rows)."""
    g = torch.Generator().manual_seed(7 + seg)
    feats = torch.randn(BFULL, T, 80, generator=g)
    tok = torch.randint(1, V, (BFULL, U), generator=g)
    tl = [U, 97, 131, 64]
    return feats, tok, tl


def main():
    rank, world, port, acc, out = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]),
                                   int(sys.argv[4]), sys.argv[5])
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    if world > 1:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
    import statecatcher_amd.train as train_mod
    from statecatcher_amd.model import ASRModel, CTCLoss, build_lucyrnn_config
    from statecatcher_amd.train import SegmentTrainer
    first_grads = []
    orig_step = train_mod.clip_and_adam_step

    def capture(opt, params, max_norm):   # the all-reduced gradients of the first update
        if not first_grads:
            first_grads.extend(p.grad.detach().float().cpu().clone() for p in params)
        return orig_step(opt, params, max_norm)
    train_mod.clip_and_adam_step = capture
    torch.manual_seed(11 + 1000 * rank)
    model = ASRModel(None, build_lucyrnn_config(80, 512, 6, V), vocab_size=V, feat_dim=80,
                     proj_dim=-1).to(dev)
    with torch.no_grad():
        model.encoder.output_proj.weight.normal_(0, 0.02)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):   # images of OWN weights
        model(torch.randn(1, 64, 80, device=dev), torch.ones(1, 64, dtype=torch.bool, device=dev))
    params = list(model.parameters())
    opt = torch.optim.Adam(params, lr=3e-4)
    tr = SegmentTrainer(model, CTCLoss(blank=0, zero_infinity=True), opt, amp_dtype=torch.bfloat16,
                        max_grad_norm=50.0, bucket_cap_mb=8.0, accumulation_steps=acc,
                        ddp=world > 1)
    if world > 1:
        assert isinstance(tr.net, torch.nn.parallel.DistributedDataParallel)
        assert tr.net.bucket_bytes_cap == 8 * 1024 * 1024
    B = BFULL // world
    rows = slice(rank * B, (rank + 1) * B)
    tr.begin_batch()
    losses, equal = [], []
    for seg in range(SEGS):
        feats, tok, tl = batch(seg)
        loss = tr.train_segment(feats[rows].to(dev), torch.ones(B, T, dtype=torch.bool, device=dev),
                                tok[rows].to(dev), [T] * B, tl[rows])
        losses.append(float(loss.detach()))
        if world > 1:
            flat = torch.cat([p.detach().reshape(-1) for p in params])
            got = [torch.empty_like(flat) for _ in range(world)]
            dist.all_gather(got, flat)
            equal.append(all(torch.equal(got[0], x) for x in got[1:]))
    torch.cuda.synchronize()
    res = {"losses": losses, "ranks_bitwise_equal": equal}
    if rank == 0:
        res["params"] = [p.detach().cpu() for p in params]
        res["grads"] = first_grads
    torch.save(res, out)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
