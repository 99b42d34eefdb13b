#!/usr/bin/env python3
"""Streaming decode throughput/latency on one GPU.

Native LucyRNN 6 x 512, 80-d input, V = 1024 (the C2 shape, infer mode), B concurrent streams:
  * statecatcher_amd.StreamingLucyRNN: hipGraph per block of K frames (and eager for contrast),
    fp32 and bf16;
  * the reference-structured eager loop (LucyRNN.step: lucyrnn.py:174-182 with torch ops per
    layer) + torch.argmax, i.e. what the reference does per frame on a GPU.
Prints one JSON object per configuration: stream frames/s (B x frames / s) and ms per frame.

usage: python tools/stream_bench.py [--frames 256] [--batches 1,16,64,256]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, n, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--batches", default="1,16,64,256")
    ap.add_argument("--fused", type=int, default=0)
    ap.add_argument("--engines", default="frame,library")
    ap.add_argument("--dtypes", default="float32,bfloat16")
    ap.add_argument("--no-reference", action="store_true")
    ap.add_argument("--schedules", default="wavefront,frame",
                    help="frame engine block schedules (StreamingLucyRNN schedule=)")
    ap.add_argument("--ks", default="1,8", help="frames per graph call")
    args = ap.parse_args()
    import statecatcher_amd as sc
    from statecatcher_amd.streaming import StreamingLucyRNN
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = sc.LucyRNNConfig(input_dim=80, hidden_dim=512, num_layers=6, vocab_size=1024,
                           is_training=False, fused_ops=bool(args.fused))
    m = sc.LucyRNN(cfg).to(dev)
    with torch.no_grad():
        m.output_proj.weight.normal_(0.0, 0.02)
    N = args.frames
    for B in [int(b) for b in args.batches.split(",")]:
        x = torch.randn(B, N, 80, device=dev)
        kgs = [(int(k), True) for k in args.ks.split(",")] + [(1, False)]
        for engine, sched, dt, K, graph in [
                (e, sc_, getattr(torch, d)) + kg for e in args.engines.split(",")
                for sc_ in (args.schedules.split(",") if e == "frame" else ["frame"])
                for d in args.dtypes.split(",") for kg in kgs]:
                if sched == "wavefront" and K == 1:
                    continue   # (one frame per block: the same launches as "frame")
                st = StreamingLucyRNN(m, B, K, dtype=dt, graph=graph, engine=engine,
                                      schedule=sched)
                blocks = [x[:, i:i + K].contiguous() for i in range(0, N, K)]
                it = iter(range(10 ** 9))

                def run():
                    st.step(blocks[next(it) % len(blocks)])
                nb = N // K
                dt_s = timed(run, nb)
                print(json.dumps({"impl": f"hip_{engine}" + (f"_{sched}" if engine == "frame" else "")
                                  + ("_graph" if graph else "_eager"),
                                  "dtype": str(dt).split(".")[-1], "B": B, "K": K,
                                  "fused": args.fused, "frames": nb * K,
                                  "stream_frames_per_s": round(B * nb * K / dt_s, 1),
                                  "ms_per_frame": round(1e3 * dt_s / (nb * K), 4)}), flush=True)
        if args.no_reference:
            continue
        # reference-structured eager per-frame loop (fp32), argmax per frame
        states = ([torch.zeros(B, 512, device=dev) for _ in range(6)],
                  [torch.zeros(B, 512, device=dev) for _ in range(6)])
        ref_state = [states]
        fr = iter(range(10 ** 9))

        @torch.no_grad()
        def ref():
            lg, ref_state[0] = m.step(x[:, next(fr) % N], ref_state[0])
            torch.argmax(lg, -1)
        n_ref = min(N, 128)
        dt_s = timed(ref, n_ref)
        print(json.dumps({"impl": "torch_eager_reference_loop", "dtype": "float32", "B": B,
                          "K": 1, "fused": args.fused, "frames": n_ref,
                          "stream_frames_per_s": round(B * n_ref / dt_s, 1),
                          "ms_per_frame": round(1e3 * dt_s / n_ref, 4)}), flush=True)


if __name__ == "__main__":
    main()
