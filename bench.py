#!/usr/bin/env python3
"""LucyRNN + CTC stateful training step on MI355X: audio-frames/sec (BASELINE.json metric).

Workload (BASELINE.json configs[1]): LucyRNN 6 x 512, 80-d synthetic fbank,
B=32 per GPU, T=1500 frames per segment, V=1024, CTC (blank 0, mean, zero_infinity),
bf16 autocast GEMMs + bf16 gates (fp32 recurrent state), Adam lr 3e-4, clip_grad_norm 50,
4 consecutive segments per batch with the encoder state carried (detached) between them.
One step = forward + CTC + backward + (DDP all-reduce) + clip + Adam over one B x T segment.

    python bench.py [--gpus N --steps K --warmup W]   (N > 1: spawns N rank processes itself)
    torchrun --nproc-per-node N ... bench.py --gpus N   (one rank per GPU, RCCL)

Prints ONE JSON line on rank 0.  value = frames processed by all ranks / max-over-ranks time.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
PEAK_BF16_TFLOPS = 2500.0  # dense bf16 MFMA spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--workload", choices=["ctc", "rnnt", "xlstm"], default="ctc",
                    help="ctc: C2/C3 LucyRNN 6x512 + CTC (the BASELINE metric); rnnt: C5 LucyRNN "
                         "6x512 + RNN-T (fused joiner, U=150); xlstm: C4 xLSTM 12 x 768 + CTC")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=1500)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--hidden", type=int, default=512)
    ap.add_argument("--vocab", type=int, default=1024)
    ap.add_argument("--feat", type=int, default=80)
    ap.add_argument("--segments", type=int, default=4)
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16")
    ap.add_argument("--output-head", choices=["split", "bf16"], default="split",
                    help="CTC workload under bf16: 'split' = the output projection as one bf16 GEMM "
                         "on split-precision operands with fp32 logits (ops.CTCHeadFn: gradients "
                         "match the fp32 oracle); 'bf16' = plain bf16 operands and logits")
    ap.add_argument("--bucket-mb", type=float, default=8.0,
                    help="DDP gradient bucket size: ~one layer (7.3 MB fp32) per bucket, so each "
                         "layer's all-reduce overlaps the backward of the layers below it")
    ap.add_argument("--cpu-baseline", choices=["on", "off"], default="on")
    ap.add_argument("--cpu-seq", type=int, default=1500,
                    help="T of the bounded CPU sample (default: one full C2 segment, ~10 s)")
    ap.add_argument("--tunableop", choices=["on", "off"], default="on",
                    help="use the shipped PyTorch TunableOp GEMM table (statecatcher_amd/tuning)")
    ap.add_argument("--timing-steps", type=int, default=2,
                    help="per-kernel HIP-event timing is recorded over the last N timed steps (each "
                         "event pair idles the GPU ~6 us; timing every step would tax the step time)")
    ap.add_argument("--host-probe", action="store_true",
                    help="diagnostics on stderr: synchronising ops in one step (sync debug mode) and "
                         "host issue time per step")
    ap.add_argument("--optimizer", choices=["hip", "torch-fused"], default="hip",
                    help="hip: torch.optim.Adam stepped by the HIP clip+Adam kernels (default); "
                         "torch-fused: torch's fused Adam kernel (A/B)")
    ap.add_argument("--graph", choices=["on", "off"], default="off",
                    help="on: each segment position's forward + backward captured once as a HIP "
                         "graph and replayed (graphs.GraphedSegments; clip + Adam eager); the "
                         "per-kernel roofline timing then comes from --timing-steps eager steps "
                         "right after the timed region (events are not recorded by a replay)")
    ap.add_argument("--op-probe", action="store_true",
                    help="diagnostics on stderr: every ATen op one step dispatches (count, shapes, "
                         "caller), to find the step's non-HIP kernels")
    ap.add_argument("--rccl-footprint", default=None, metavar="WGS[:SLEEP]",
                    help="diagnostic (1 GPU): mimic a DP all-reduce's footprint -- during the "
                         "backward, as each large gradient is produced, WGS persistent workgroups "
                         "on a side stream copy 2 (8 - 1) / 8 of its bytes (an 8-GPU ring's share), "
                         "paced by SLEEP; the optimizer step waits for them, as DDP's does "
                         "(tools/footprint.hip, built by tools/footprint.sh)")
    ap.add_argument("--tune-out", default=None,
                    help="rank 0 tunes GEMM shapes missing from the table and writes it here")
    ap.add_argument("--retune", action="store_true",
                    help="with --tune-out: ignore the shipped table and tune every shape afresh "
                         "(1 s budget per shape)")
    return ap.parse_args()


def synth_segments(args, rank, device):
    g = torch.Generator().manual_seed(1234 + rank)
    gt = torch.Generator().manual_seed(4321 + rank)
    segs = []
    for _ in range(args.segments):
        feats = torch.randn(args.batch, args.seq, args.feat, generator=g)
        U = torch.randint(50, 151, (args.batch,), generator=gt)
        if args.workload == "rnnt":   # U = 150 for C5
            U = torch.full((args.batch,), 150, dtype=torch.int64)
        tok = torch.randint(1, args.vocab, (args.batch, 150), generator=gt)
        for b in range(args.batch):
            tok[b, U[b]:] = 0
        segs.append(dict(feats=feats.to(device), tokens=tok.to(device),
                         in_lens=torch.full((args.batch,), args.seq, dtype=torch.int64, device=device),
                         tgt_lens=U.to(device),
                         masks=torch.ones(args.batch, args.seq, dtype=torch.bool, device=device)))
    return segs


def gemm_flops_per_frame(args):
    if args.workload == "xlstm":
        return None
    D, L = args.hidden, args.layers
    fwd = 2 * 7 * D * (args.feat + (L - 1) * D) + 2 * D * args.vocab
    return 3 * fwd   # fwd + dgrad + wgrad


def op_probe(step):
    """Run one step under a TorchDispatchMode and print the ATen ops that launch work (views and
    metadata ops excluded), grouped by op, shapes and the innermost statecatcher_amd caller."""
    import collections
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    skip = ("view", "_unsafe_view", "t", "transpose", "permute", "expand", "slice", "select",
            "as_strided", "detach", "alias", "unsqueeze", "squeeze", "split", "empty", "split_with_sizes",
            "_reshape_alias", "reshape", "unbind", "chunk", "is_same_size", "_to_copy_meta",
            "empty_strided", "new_empty", "new_empty_strided", "narrow", "lift_fresh", "_local_scalar_dense")
    seen = collections.Counter()

    class Mode(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = func.overloadpacket.__name__
            if name not in skip:
                shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))[:3]
                where = "?"
                for fr in reversed(traceback.extract_stack()[:-1]):
                    if "statecatcher_amd" in fr.filename or fr.filename.endswith("bench.py"):
                        where = f"{os.path.basename(fr.filename)}:{fr.lineno}"
                        break
                seen[(name, shapes, where)] += 1
            return func(*args, **(kwargs or {}))

    torch.cuda.synchronize()
    with Mode():
        step()
    torch.cuda.synchronize()
    for (name, shapes, where), n in sorted(seen.items(), key=lambda kv: kv[0][2]):
        print(f"op-probe {n:3d}x {name:28s} {where:28s} {shapes}", file=sys.stderr)


def build_workload(args, device):
    """(model, criterion, optimizer params, trainer kwargs, config dict) per workload."""
    from statecatcher_amd.model import (ASRModel, CTCLoss, RNNTLoss, RNNTPredictorJoiner,
                                        build_lucyrnn_config, build_xlstm_config)
    torch.manual_seed(0)   # identical init on every rank (DDP also broadcasts)
    if args.workload == "xlstm":
        # C4: xLSTM-large 12 blocks x 768 (4 heads: DQK 96, DV 192) behind the 80 -> 768 input
        # projection, CTC; T padded to the 64-step chunk inside ASRModel (model.py:341-347)
        cfg = build_xlstm_config(args.feat, args.vocab, num_heads=4, num_blocks=12, embedding_dim=768)
        model = ASRModel(None, cfg, vocab_size=args.vocab, feat_dim=args.feat, proj_dim=-1).to(device)
        conf = {"workload": "xLSTM 12x768 (mLSTM, 4 heads) + CTC training step, stateful "
                            f"{args.segments}-segment carry", "blocks": 12, "embedding_dim": 768,
                "mlstm_cell_dtype": cfg.autocast_kernel_dtype}   # float16 as model.py:227
        return model, CTCLoss(blank=0, zero_infinity=True), list(model.parameters()), \
            dict(mode="ctc"), conf
    cfg = build_lucyrnn_config(args.feat, args.hidden, args.layers, args.vocab)
    model = ASRModel(None, cfg, vocab_size=args.vocab, feat_dim=args.feat, proj_dim=-1).to(device)
    with torch.no_grad():   # reference zero-inits output_proj (lucyrnn_triton.py:108-109); a seeded
        model.encoder.output_proj.weight.normal_(0, 0.02)   # N(0,0.02) keeps every gradient non-zero
    conf = {"layers": args.layers, "hidden": args.hidden}
    if args.workload == "rnnt":
        # C5: RNNTPredictorJoiner(enc_out_dim=V, 64, 64, V) (train.py:368-375, :638-639), trained
        # by the same optimizer; clip covers the model only (train.py:553)
        joiner = RNNTPredictorJoiner(args.vocab, 64, 64, args.vocab).to(device)
        conf["workload"] = (f"LucyRNN {args.layers}x{args.hidden} + RNN-T (fused joiner, J=64, "
                            f"U=150) training step, stateful {args.segments}-segment carry")
        return model, RNNTLoss(blank=0), list(model.parameters()) + list(joiner.parameters()), \
            dict(mode="rnnt", joiner=joiner), conf
    conf["workload"] = (f"LucyRNN {args.layers}x{args.hidden} + CTC training step, stateful "
                        f"{args.segments}-segment carry")
    split = args.output_head == "split"
    if args.dtype == "bf16":
        from statecatcher_amd import ops as _ops
        conf["output_projection"] = (
            {"emis": "bf16 GEMM and logits; the lattice's emission columns to fp32 accuracy from "
                     "split-precision operands (side array)",
             "labels": "bf16 GEMM on split-precision operands, fp32 logits",
             "full": "split-precision GEMM, fp32 logits"}.get(_ops.HEAD_SPLIT, _ops.HEAD_SPLIT)
            if split else "bf16 operands and logits")
    return model, CTCLoss(blank=0, zero_infinity=True, fused_head=split), list(model.parameters()), \
        dict(mode="ctc"), conf


def footprint_hooks(model, spec, device):
    """bench --rccl-footprint: per large gradient, a side-stream copy of 2 (N - 1) / N of its
    bytes at N = 8 by `wgs` workgroups (RCCL's ring kernels hold a few dozen CUs for the whole
    all-reduce); the main stream waits for the side stream once the last gradient is in (DDP's
    wait before the optimizer step).  Returns the side stream."""
    import ctypes
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "ab", "footprint", "libfootprint.so"))
    lib.sc_probe_footprint.restype = ctypes.c_int
    lib.sc_probe_footprint.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    wgs, _, sleep = spec.partition(":")
    wgs, sleep = int(wgs), int(sleep or 0)
    big = [p for p in model.parameters() if p.numel() >= 1 << 20]
    nbytes = max(p.numel() for p in big) * 4 * 2
    src = torch.empty(nbytes // 4, device=device)
    dst = torch.empty_like(src)
    side = torch.cuda.Stream(device)

    def launch(p):
        b = int(2 * 7 / 8 * p.numel() * 4) // 16 * 16
        side.wait_stream(torch.cuda.current_stream(device))
        rc = lib.sc_probe_footprint(src.data_ptr(), dst.data_ptr(), b, wgs, sleep,
                                    ctypes.c_void_p(side.cuda_stream))
        assert rc == 0, rc

    for p in big:
        p.register_post_accumulate_grad_hook(launch)
    # the input projection's weight gradient is the backward's last large one
    last = model.encoder.tracks[0][0].linear.weight if hasattr(model.encoder, "tracks") else big[0]
    last.register_post_accumulate_grad_hook(
        lambda p: torch.cuda.current_stream(device).wait_stream(side))
    return side


def cpu_quota():
    """This process's CPU allowance: the cgroup v2 quota (cpu.max "quota period" -> CPUs), the
    affinity mask and OMP_NUM_THREADS, as a string for the cpu_baseline record."""
    parts = []
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        parts.append("cgroup cpu.max " + ("unlimited" if q == "max" else
                                          f"{int(q) / int(per):g} CPUs ({q}/{per})"))
    except Exception:
        parts.append("cgroup cpu.max unreadable")
    try:
        parts.append(f"affinity {len(os.sched_getaffinity(0))} CPUs")
    except Exception:
        pass
    parts.append(f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS', 'unset')}")
    return ", ".join(parts)


def cpu_baseline(args):
    """Oracle (numpy port) of the same step on a bounded sample: B=32, T=args.cpu_seq."""
    from oracle import lucy_step
    try:
        from threadpoolctl import threadpool_info
        threads = max([i.get("num_threads", 1) for i in threadpool_info()] or [1])
    except Exception:   # pragma: no cover
        threads = 1
    B, T = args.batch, args.cpu_seq
    rng = np.random.default_rng(0)
    p = lucy_step.init_params(args.layers, args.feat, args.hidden, args.vocab)
    feats = rng.standard_normal((B, T, args.feat)).astype(np.float32)
    U = rng.integers(max(1, T // 30), max(2, T // 10) + 1, B)
    tok = rng.integers(1, args.vocab, (B, int(U.max())))
    in_lens = np.full(B, T)
    t0 = time.perf_counter()
    loss, state, _, adam = lucy_step.train_step(p, feats, tok, in_lens, U, args.layers, args.hidden)
    dt = time.perf_counter() - t0
    model = cpu_model()
    return {"value": round(B * T / dt, 1), "unit": "audio-frames/s", "cores": int(threads),
            "kind": "port",
            "sample": f"oracle/lucy_step.py numpy fp32 (CTC fp64) train step, B={B} T={T} "
                      f"(U~[{T // 30},{T // 10}]), {args.layers}x{args.hidden}, 1 step, "
                      f"{dt:.1f} s on {model} (os.cpu_count={os.cpu_count()}, BLAS threads="
                      f"{threads} = this job's CPU share)",
            "cpu_quota": cpu_quota(),
            "c1_nn_lstm": c1_lstm_baseline()}


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:   # pragma: no cover
        pass
    return platform.processor() or platform.machine()


def c1_lstm_baseline(seconds=4.0):
    """BASELINE.json configs[0] (C1): torch.nn.LSTM(80, 256, 2) + Linear(256 -> 1024) +
    nn.CTCLoss(blank=0, zero_infinity=True), fwd + bwd + Adam, B=4, T=200, on the host CPU with
    torch's intra-op threads (model.py:203-212, train.py:142).  Pure PyTorch, not reference code."""
    import torch.nn as nn
    g = torch.Generator().manual_seed(7)
    B, T, V = 4, 200, 1024
    lstm = nn.LSTM(80, 256, num_layers=2, batch_first=True)
    cls = nn.Linear(256, V)
    crit = nn.CTCLoss(blank=0, zero_infinity=True)
    opt = torch.optim.Adam(list(lstm.parameters()) + list(cls.parameters()), lr=3e-4)
    feats = torch.randn(B, T, 80, generator=g)
    U = torch.randint(5, 21, (B,), generator=g)
    tok = torch.randint(1, V, (B, 20), generator=g)

    def step():
        out, _ = lstm(feats)
        loss = crit(cls(out).log_softmax(-1).transpose(0, 1), tok, [T] * B, U.tolist())
        opt.zero_grad()
        loss.backward()
        opt.step()

    step()   # warm-up (first call allocates)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        step()
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * B * T / dt, 1), "unit": "audio-frames/s",
            "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"C1 nn.LSTM 2x256 + Linear + CTC fwd+bwd+Adam, B={B} T={T}, {n} steps in "
                      f"{dt:.1f} s, torch CPU threads={torch.get_num_threads()}"}


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n, port, base=None):
    """torchrun's per-rank environment for n ranks on this node (rendezvous on 127.0.0.1)."""
    base = dict(os.environ if base is None else base)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL on this host
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        envs.append(e)
    return envs


def spawn_ranks(n, cmd, port=None):
    """Run `cmd` as n child processes, one per GPU rank, and return the first non-zero exit
    code (0 if all ranks succeed).  The parent never initialises HIP: children are started as
    new processes (no fork of a HIP context, no exec of this one).  If a rank fails the others
    are terminated, so a hung collective cannot outlive the failure."""
    import subprocess
    port = port or free_port()
    procs = [subprocess.Popen(cmd, env=e) for e in rank_envs(n, port)]
    rc = 0
    try:
        pending = set(range(n))
        while pending:
            for r in sorted(pending):
                code = procs[r].poll()
                if code is None:
                    continue
                pending.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:
                        procs[q].terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def count_gpus_without_hip(topo="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs this process may use, counted WITHOUT touching HIP: the parent forks and execs the
    rank processes, and HIP initialised before a fork/exec is unusable in the children (and on
    this pool an exec after GPU initialisation takes the machine down).  torch.cuda.device_count()
    tries amdsmi but falls back to hipGetDeviceCount, so it is not used here.  Sources, in order:
    the KFD topology in sysfs (nodes with SIMDs are GPUs), then amdsmi; a HIP_VISIBLE_DEVICES /
    ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES list caps the count.  None when neither source
    answers."""
    n = None
    try:
        n = 0
        for node in os.listdir(topo):
            with open(os.path.join(topo, node, "properties")) as f:
                props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except (OSError, ValueError):
        n = None
    if not n:
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            try:
                n = len(amdsmi.amdsmi_get_processor_handles())
            finally:
                amdsmi.amdsmi_shut_down()
        except Exception:
            n = None
    if n is None:
        return None
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def main():
    args = parse()
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1, got {args.gpus}")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # plain `python bench.py --gpus N`: start N ranks ourselves (torchrun's environment)
        ndev = count_gpus_without_hip()
        if ndev is None:
            sys.exit("bench.py: cannot count GPUs without initialising HIP (no KFD topology in "
                     "sysfs, no amdsmi); launch the ranks with torchrun instead")
        if ndev < args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but only {ndev} GPU(s) visible")
        sys.exit(spawn_ranks(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} does not match --gpus {args.gpus}")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    if args.tunableop == "on":
        # hipBLASLt/rocBLAS solution table for this model's GEMM shapes (tools/blas_probe.py):
        # the default heuristics pick e.g. 263 us for the gate GEMM that a tuned solution does
        # in 146 us.  Tuning itself only ever runs in warmup, and only with --tune-out.
        import torch.cuda.tunable as tun
        table = os.path.join(ROOT, "statecatcher_amd", "tuning", "tunableop_gfx950.csv")
        tun.enable(True)
        tun.tuning_enable(bool(args.tune_out) and rank == 0)
        tun.set_max_tuning_duration(1000 if args.retune else 200)
        tun.set_filename(args.tune_out if (args.tune_out and rank == 0) else table)
        if os.path.exists(table) and not (args.retune and args.tune_out):
            tun.read_file(table)

    from statecatcher_amd import ops
    from statecatcher_amd.train import SegmentTrainer

    model, criterion, params, tkw, conf = build_workload(args, device)
    params = [p for p in params if p.requires_grad]
    if args.optimizer == "torch-fused":   # A/B: torch's fused Adam with the clip as grad_scale
        opt = torch.optim.Adam(params, lr=3e-4, fused=True)
    else:   # the reference's optim.Adam(params, lr) (train.py:133): clip + step on HIP (optim.py)
        opt = torch.optim.Adam(params, lr=3e-4)
    amp = torch.bfloat16 if args.dtype == "bf16" else None
    # the reference segment loop (train.py:460-581) with DDP over RCCL when world > 1
    # --graph on: no DDP wrapper; the graphs broadcast rank 0's weights and all-reduce the
    # gradients after each replay themselves (graphs.GraphedSegments)
    trainer = SegmentTrainer(model, criterion, opt, accumulation_steps=1, max_grad_norm=50.0,
                             amp_dtype=amp, bucket_cap_mb=args.bucket_mb,
                             ddp=(world > 1 and args.graph != "on"), **tkw)
    segs = synth_segments(args, rank, device)
    if args.rccl_footprint:
        footprint_hooks(model, args.rccl_footprint, device)

    def eager_step():
        i = trainer.global_step
        if i % args.segments == 0:
            trainer.begin_batch()   # new batch: state reset (train.py:460)
        seg = segs[i % args.segments]
        return trainer.train_segment(seg["feats"], seg["masks"], seg["tokens"], seg["in_lens"],
                                     seg["tgt_lens"])

    step = eager_step
    # (data-parallel graph mode: no eager warm-up -- without the DDP wrapper its steps would not
    # all-reduce; the capture warms up on its own and the replays below warm the graphs)
    for _ in range(args.warmup if not (args.graph == "on" and world > 1) else 0):
        step()
    torch.cuda.synchronize()
    graphed = None
    if args.graph == "on":
        # world > 1: the graphs hold each rank's forward + backward, the gradients are
        # all-reduced after every replay (graphs.GraphedSegments)
        from statecatcher_amd.graphs import GraphedSegments
        graphed = GraphedSegments(trainer, segs).capture()

        def step():
            if trainer.global_step % args.segments == 0:
                graphed.begin_batch()
            return graphed.step()
        if args.warmup:
            for _ in range(max(args.segments, args.warmup if world > 1 else 0)):
                step()   # one replay of every graph (data parallel: the warm-up steps) before timing
        torch.cuda.synchronize()
    if args.host_probe:
        torch.cuda.set_sync_debug_mode(1)
        step()
        torch.cuda.set_sync_debug_mode(0)
        torch.cuda.synchronize()
        for _ in range(3):
            h0 = time.perf_counter()
            step()
            h1 = time.perf_counter()
            torch.cuda.synchronize()
            h2 = time.perf_counter()
            print(f"host issue {1e3 * (h1 - h0):.3f} ms, step wall {1e3 * (h2 - h0):.3f} ms",
                  file=sys.stderr)
    if args.op_probe:
        op_probe(step)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        if graphed is None and k == max(0, args.steps - args.timing_steps):
            ops.LAUNCH_EVENTS = []
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    last_loss = float(loss.item())
    if graphed is not None and args.timing_steps > 0:
        # a replay records no per-launch events: the kernel timings come from eager steps of the
        # same segments right after the timed region (same kernels, same shapes)
        for p in graphed.params:
            p.grad = None
        ops.LAUNCH_EVENTS = []
        for _ in range(args.timing_steps):
            eager_step()
        torch.cuda.synchronize()
    events, ops.LAUNCH_EVENTS = ops.LAUNCH_EVENTS or [], None

    # per-kernel average launch duration from the HIP events recorded on the launch stream
    kstats = {}
    for name, e0, e1, nbytes, flops in events:
        k = kstats.setdefault(name, [0.0, 0, 0, 0])
        k[0] += e0.elapsed_time(e1) * 1e-3
        k[1] += 1
        k[2] = nbytes
        k[3] += flops
    kernels = {}
    for name, (tsum, n, nbytes, _) in kstats.items():
        avg = tsum / n
        tsteps = max(1, min(args.timing_steps, args.steps))
        kernels[name] = {"launches": n, "avg_us": round(avg * 1e6, 1),
                         "share_of_step": round(tsum / tsteps / (dt / args.steps), 4)}
        if nbytes:
            kernels[name].update({"bytes_per_launch": nbytes,
                                  "achieved_GBs": round(nbytes / avg / 1e9, 1),
                                  "frac_of_peak": round(nbytes / avg / 1e9 / PEAK_HBM_GBS, 4)})
    scans = [k for k in kernels if k.startswith("lucy_scan") or k.startswith("mlstm")]
    dom = max(scans, key=lambda k: kstats[k][0]) if scans else None
    # PMC-measured HBM bytes per launch of that kernel, from the rocprofv3 passes of a bench run
    # of THIS workload and dtype (tools/pmc_traffic.py keys them "<workload>/<dtype>"); null when
    # no such pass was taken
    traffic = None
    pmc_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    pmc_key = f"{args.workload}/{'bf16' if args.dtype == 'bf16' else 'fp32'}"
    if dom and os.path.exists(pmc_file):
        traffic = json.load(open(pmc_file)).get(pmc_key, {}).get(dom, {}).get("hbm_bytes_per_launch")
    roofline = None
    if dom:
        kd = kernels[dom]
        roofline = {"bound": "hbm", "kernel": dom, "achieved": kd["achieved_GBs"],
                    "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": kd["frac_of_peak"],
                    "traffic": traffic}
    # C5: the fused joiner owns half the step and is MFMA work.  Per launch (one segment of B
    # sequences, all T = seq frames, U + 1 = 151 label positions): N = B T (U+1) lattice nodes,
    # joint_fwd 2 N V J flops (the logits once), joint_bwd 3 x 2 N V J (logits recomputed, dW,
    # dZ); J = 64.  Peak: bf16 dense MFMA (MI355X_MICROARCH.md).
    # C4: the step belongs to its GEMMs (the xLSTM block linears: forward, input and weight
    # gradients; profiles/r3d_prof_xlstm.md), so the roofline is theirs, as one class: the flops
    # of every timed GEMM launch over their summed HIP-event time, against the bf16 MFMA peak
    if args.workload == "xlstm" and "xlstm_gemm" in kstats:
        tsum, n, _, fl = kstats["xlstm_gemm"]
        tfs = fl / tsum / 1e12
        kernels["xlstm_gemm"].update({"flops_per_step": fl / max(1, min(args.timing_steps, args.steps)),
                                      "achieved_TFLOPs": round(tfs, 1),
                                      "frac_of_peak": round(tfs / PEAK_BF16_TFLOPS, 4)})
        roofline = {"bound": "mfma", "kernel": "xlstm_gemm (all block linears: fwd, dX, dW)",
                    "achieved": round(tfs, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(tfs / PEAK_BF16_TFLOPS, 4), "traffic": None,
                    "mlstm": {k: kernels[k] for k in ("mlstm_fwd", "mlstm_bwd") if k in kernels}}
    if args.workload == "rnnt":
        nodes = args.batch * args.seq * 151
        for name, mult in (("rnnt_joint_fwd", 1), ("rnnt_joint_bwd", 3)):
            if name in kernels:
                fl = mult * 2.0 * nodes * args.vocab * 64
                tfs = fl / (kernels[name]["avg_us"] * 1e-6) / 1e12
                kernels[name].update({"flops_per_launch": fl, "achieved_TFLOPs": round(tfs, 1),
                                      "frac_of_peak": round(tfs / PEAK_BF16_TFLOPS, 4)})
        if "rnnt_joint_bwd" in kernels:
            kj = kernels["rnnt_joint_bwd"]
            roofline = {"bound": "mfma", "kernel": "rnnt_joint_bwd", "achieved": kj["achieved_TFLOPs"],
                        "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": kj["frac_of_peak"],
                        "traffic": None}

    frames = world * args.batch * args.seq * args.steps
    value = frames / dt
    ms = dt / args.steps * 1e3
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "on" and args.workload == "ctc":
        cpu = cpu_baseline(args)
    if rank == 0:
        gf = gemm_flops_per_frame(args)
        gemm_tflops = gf * args.batch * args.seq * world * args.steps / dt / 1e12 if gf else None
        line = {
            "metric": {"ctc": "audio-frames/sec (LucyRNN+CTC, 80-d fbank, T=1500), whole job",
                       "rnnt": "audio-frames/sec (LucyRNN+RNN-T, 80-d fbank, T=1500, U=150), whole job",
                       "xlstm": "audio-frames/sec (xLSTM+CTC, 80-d fbank, T=1500), whole job"}[args.workload],
            "value": round(value, 1), "unit": "audio-frames/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if amp is not None else "fp32",
            "data": "synthetic N(0,1) 80-d fbank, targets " +
                    ("U=150" if args.workload == "rnnt" else "U~U[50,150]") +
                    " of V=1024, random-init weights",
            "config": {**conf, "global_batch": args.batch * world, "seq_len": args.seq,
                       "vocab": args.vocab, "parallelism": f"dp{world}"},
            "per_gpu_frames_per_s": round(value / world, 1),
            "roofline": roofline,
            "kernels": kernels,
            "kernel_timing": (f"HIP events on the launch stream, last {min(args.timing_steps, args.steps)} "
                              "timed steps") if graphed is None else
                             (f"HIP events on the launch stream, {args.timing_steps} eager steps "
                              "right after the timed graph replays"),
            "launch": "hip-graph replay per segment (forward + backward), clip + Adam eager"
                      if graphed is not None else "eager",
            "gemm_TFLOPs_effective": round(gemm_tflops / world, 1) if gemm_tflops else None,
            "cpu_baseline": cpu,
            "loss_last": round(last_loss, 4),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
