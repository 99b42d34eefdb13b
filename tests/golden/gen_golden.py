#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.npz from the REFERENCE itself.

Runs only in the build container (needs /root/reference; never on the GPU box):

    TRITON_INTERPRET=1 python tests/golden/gen_golden.py

Sources of truth, per fixture file:
  scan_fwd.npz     reference Triton kernel ``rnn_forward_unfused_rmsnorm``
                   (lucyrnn_triton.py:179-244) executed by the Triton CPU interpreter, fp32.
  scan_bwd.npz     no reference backward exists: torch.autograd of an fp64
                   restatement of the forward (whose outputs are checked against
                   scan_fwd.npz by tests/test_oracle_golden.py).
  decay_scan.npz   reference Triton kernel ``fused_decay_scan`` (lucyrnn_triton.py:158-177).
  ctc.npz          ATen ``torch.ctc_loss`` (CPU fp64), the op behind the reference's
                   ``nn.CTCLoss(blank=0, zero_infinity=True)`` (train.py:142, model.py:68-71).
  greedy.npz       reference ``decoder.ctc_greedy_decoder`` (decoder.py:3-30).
  native.npz       reference ``lucyrnn.LucyRNN`` (lucyrnn.py:72-191), train and infer modes.
  module.npz       reference ``lucyrnn_triton.LucyRNNtriton`` (lucyrnn_triton.py:77-155) at its
                   own init, fp32, Triton interpreter: 3 layers with the inter-layer LayerNorms
                   and output_proj, two segments with the state carried (h made contiguous
                   between them).

Only arrays are stored (np.savez, allow_pickle not needed).  Seeds are fixed below.
"""
import os
import sys

os.environ.setdefault("TRITON_INTERPRET", "1")
os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.dont_write_bytecode = True
sys.path.insert(0, REF)


def ref_scan_fwd(gates, h0, s0):
    from lucyrnn_triton import rnn_forward_unfused_rmsnorm
    gates = gates.contiguous()
    B, T, _, D = gates.shape
    out = torch.empty(B, T, D, dtype=gates.dtype)
    s_out = torch.empty(B, D, dtype=gates.dtype)
    # launch exactly as lucyrnn_triton.py:61-73 does
    rnn_forward_unfused_rmsnorm[(B, D)](
        gates_ptr=gates, h0_ptr=h0, s0_ptr=s0, out_ptr=out, s_out_ptr=s_out,
        B=B, T=T, D=D,
        stride_g_bt=gates.stride(0), stride_g_td=gates.stride(1), stride_g_cd=gates.stride(2),
        stride_o_bt=out.stride(0), stride_o_bd=out.stride(1))
    return out, s_out


def torch_scan_fwd64(gates, h0, s0):
    """fp64 restatement used only to obtain autograd gradients (SURVEY §8c backward oracle)."""
    eps = 1e-6
    B, T, _, D = gates.shape
    h, s = h0, s0
    outs = []
    for t in range(T):
        r, z, k, v, hp, dc, al = [gates[:, t, i] for i in range(7)]
        rc = torch.sqrt((r * r + z * z) / 2 + eps)
        rkv = torch.sqrt((k * k + v * v) / 2 + eps)
        rd = torch.sqrt(dc * dc + eps)
        ra = torch.sqrt(al * al + eps)
        rh = torch.sqrt(hp * hp + eps)
        zg = torch.sigmoid(z / rc)
        dec = torch.sigmoid(dc / rd)
        alp = torch.sigmoid(al / ra)
        hn = hp / rh
        kv = (k / rkv) * (v / rkv) / (rkv * rkv + eps)
        s = dec * s + alp * kv
        c = torch.sigmoid(2 * (hn + s)) * 2 - 1
        h = (1 - zg) * c + zg * h
        outs.append(h)
    return torch.stack(outs, 1), s


def realistic_gates(B, T, Din, D, seed):
    """Gates from a reference LucyRNNCellTriton linear (xavier + gate biases, :35-48)."""
    from lucyrnn_triton import LucyRNNCellTriton
    torch.manual_seed(seed)
    cell = LucyRNNCellTriton(Din, D)
    x = torch.randn(B, T, Din)
    with torch.no_grad():
        g = cell.linear(x).view(B, T, 7, D).contiguous()
    return g


def gen_scan():
    cases = {}
    g = torch.Generator().manual_seed(1234)

    def add(name, gates, h0, s0):
        out, s_out = ref_scan_fwd(gates, h0, s0)
        cases[name + "/gates"] = gates.numpy()
        cases[name + "/h0"] = h0.numpy()
        cases[name + "/s0"] = s0.numpy()
        cases[name + "/out"] = out.numpy()
        cases[name + "/s_out"] = s_out.numpy()
        print("scan", name, tuple(gates.shape), flush=True)

    B, D = 2, 16
    add("rand_T7", torch.randn(B, 7, 7, D, generator=g) * 0.5,
        torch.randn(B, D, generator=g) * 0.1, torch.randn(B, D, generator=g) * 0.1)
    add("rand_T1", torch.randn(B, 1, 7, D, generator=g) * 0.2,
        torch.zeros(B, D), torch.zeros(B, D))
    add("rand_T64", torch.randn(B, 64, 7, D, generator=g) * 0.2,
        torch.randn(B, D, generator=g) * 0.1, torch.randn(B, D, generator=g))
    gz = torch.randn(B, 16, 7, D, generator=g) * 0.3
    gz[:, :, 2] = 0.0   # exact-zero k
    gz[:, 3:9, 3] = 0.0  # exact-zero v
    add("zero_kv", gz, torch.zeros(B, D), torch.zeros(B, D))
    add("large", torch.randn(B, 16, 7, D, generator=g) * 50.0,
        torch.randn(B, D, generator=g), torch.randn(B, D, generator=g) * 10)
    add("realistic", realistic_gates(B, 48, 24, D, 7), torch.zeros(B, D), torch.zeros(B, D))
    # odd D (masking) and a long T crossing several 64-step super-chunks
    add("odd_D", torch.randn(3, 20, 7, 13, generator=g) * 0.4,
        torch.randn(3, 13, generator=g) * 0.2, torch.randn(3, 13, generator=g) * 0.2)
    add("long_T", realistic_gates(1, 300, 8, 8, 11), torch.zeros(1, 8), torch.zeros(1, 8))
    # two-segment carry with a CONTIGUOUS h0 (the corrected semantics) ...
    g1 = torch.randn(3, 12, 7, D, generator=g) * 0.3
    g2 = torch.randn(3, 12, 7, D, generator=g) * 0.3
    o1, s1 = ref_scan_fwd(g1, torch.zeros(3, D), torch.zeros(3, D))
    h_view = o1[:, -1, :]                      # lucyrnn_triton.py:135, strided view
    o2c, s2c = ref_scan_fwd(g2, h_view.contiguous(), s1)
    o2a, s2a = ref_scan_fwd(g2, h_view, s1)   # ... and the reference's aliased read (F3)
    cases.update({"carry/g1": g1.numpy(), "carry/g2": g2.numpy(), "carry/out1": o1.numpy(),
                  "carry/s1": s1.numpy(), "carry/out2_contig": o2c.numpy(),
                  "carry/s2_contig": s2c.numpy(), "carry/out2_aliased": o2a.numpy()})
    np.savez(os.path.join(HERE, "scan_fwd.npz"), **cases)

    # backward fixtures: autograd of the fp64 restatement
    bw = {}
    for name in ["rand_T7", "rand_T64", "realistic", "odd_D", "large"]:
        gates = torch.from_numpy(cases[name + "/gates"]).double().requires_grad_(True)
        h0 = torch.from_numpy(cases[name + "/h0"]).double().requires_grad_(True)
        s0 = torch.from_numpy(cases[name + "/s0"]).double().requires_grad_(True)
        out, s_last = torch_scan_fwd64(gates, h0, s0)
        gg = torch.Generator().manual_seed(99)
        dout = torch.randn(out.shape, generator=gg, dtype=torch.float64)
        ds = torch.randn(s_last.shape, generator=gg, dtype=torch.float64)
        dg, dh0, ds0 = torch.autograd.grad((out * dout).sum() + (s_last * ds).sum(), [gates, h0, s0])
        bw.update({name + "/dout": dout.numpy(), name + "/ds_last": ds.numpy(),
                   name + "/dgates": dg.numpy(), name + "/dh0": dh0.numpy(), name + "/ds0": ds0.numpy(),
                   name + "/out64": out.detach().numpy(), name + "/s_last64": s_last.detach().numpy()})
        print("scan bwd", name, flush=True)
    np.savez(os.path.join(HERE, "scan_bwd.npz"), **bw)


def gen_decay():
    from lucyrnn_triton import fused_decay_scan
    g = torch.Generator().manual_seed(77)
    cases = {}
    for name, (B, T, D) in {"small": (2, 33, 8), "t1": (1, 1, 4)}.items():
        kv = torch.randn(B, T, D, generator=g)
        decay = torch.sigmoid(torch.randn(B, T, D, generator=g))
        s_all = torch.empty_like(kv)
        fused_decay_scan[(B, D)](kv_ptr=kv, decay_ptr=decay, output_ptr=s_all, B=B, T=T, D=D,
                                 stride_b=T * D, stride_t=D, stride_d=1)   # lucyrnn.py:147-151
        cases.update({name + "/kv": kv.numpy(), name + "/decay": decay.numpy(),
                      name + "/s_all": s_all.numpy()})
    np.savez(os.path.join(HERE, "decay_scan.npz"), **cases)
    print("decay_scan done", flush=True)


def gen_ctc():
    g = torch.Generator().manual_seed(4321)
    cases = {}

    def add(name, T, B, V, in_lens, tgt_lens, targets=None, scale=1.0):
        logits = torch.randn(B, T, V, generator=g, dtype=torch.float64) * scale
        Umax = max(max(tgt_lens), 1)
        if targets is None:
            targets = torch.randint(1, V, (B, Umax), generator=g)
        targets = targets.clone()
        for b in range(B):
            targets[b, tgt_lens[b]:] = 0        # padded with blank like train.py:208
        lg = logits.clone().requires_grad_(True)
        lp = lg.log_softmax(-1).transpose(0, 1)  # model.py:70
        nll = torch.nn.functional.ctc_loss(lp, targets, in_lens, tgt_lens, blank=0,
                                           reduction="none", zero_infinity=False)
        lg2 = logits.clone().requires_grad_(True)
        loss = torch.nn.CTCLoss(blank=0, zero_infinity=True)(lg2.log_softmax(-1).transpose(0, 1),
                                                            targets, in_lens, tgt_lens)
        loss.backward()
        # per-sample gradient of nll_b wrt logits (rows of b only), zero_infinity=False
        lg3 = logits.clone().requires_grad_(True)
        nll3 = torch.nn.functional.ctc_loss(lg3.log_softmax(-1).transpose(0, 1), targets, in_lens,
                                            tgt_lens, blank=0, reduction="none", zero_infinity=True)
        nll3.sum().backward()
        cases.update({name + "/logits": logits.numpy(), name + "/targets": targets.numpy(),
                      name + "/in_lens": np.asarray(in_lens, np.int64),
                      name + "/tgt_lens": np.asarray(tgt_lens, np.int64),
                      name + "/nll": nll.detach().numpy(), name + "/mean_loss": np.float64(loss.item()),
                      name + "/mean_grad": lg2.grad.numpy(), name + "/sum_grad": lg3.grad.numpy()})
        print("ctc", name, flush=True)

    add("basic", 50, 3, 32, [50, 41, 30], [10, 7, 0])
    add("repeats", 40, 2, 8, [40, 25], [12, 9],
        targets=torch.tensor([[3, 3, 3, 1, 1, 2, 2, 2, 5, 5, 5, 5], [7, 7, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0]]))
    add("infeasible", 10, 3, 16, [10, 5, 3], [6, 5, 3],
        targets=torch.tensor([[1, 2, 3, 4, 5, 6], [1, 1, 2, 2, 3, 0], [4, 4, 4, 0, 0, 0]]))
    add("long", 200, 2, 24, [200, 177], [60, 40], scale=3.0)
    add("u_eq_t", 8, 2, 12, [8, 8], [8, 4],
        targets=torch.tensor([[1, 2, 3, 4, 5, 6, 7, 8], [2, 2, 2, 2, 0, 0, 0, 0]]))
    np.savez(os.path.join(HERE, "ctc.npz"), **cases)


def gen_greedy():
    from decoder import ctc_greedy_decoder
    g = torch.Generator().manual_seed(555)
    B, T, V = 4, 60, 12
    # quantised values force ties (first index must win), plus one NaN row
    lp = torch.randint(-4, 1, (B, T, V), generator=g).float()
    lp[1, 5, 7] = float("nan")
    in_lens = torch.tensor([60, 33, 1, 0])
    dec = ctc_greedy_decoder(lp, in_lens, blank=0)
    lens = np.array([len(d) for d in dec], np.int64)
    flat = np.array([t for d in dec for t in d], np.int64)
    lp2 = torch.randn(3, 100, 128, generator=g)
    lp2 = lp2.log_softmax(-1)
    in2 = torch.tensor([100, 75, 17])
    dec2 = ctc_greedy_decoder(lp2, in2, blank=0)
    np.savez(os.path.join(HERE, "greedy.npz"),
             ties_lp=lp.numpy(), ties_in_lens=in_lens.numpy(), ties_counts=lens, ties_tokens=flat,
             big_lp=lp2.numpy().astype(np.float32), big_in_lens=in2.numpy(),
             big_counts=np.array([len(d) for d in dec2], np.int64),
             big_tokens=np.array([t for d in dec2 for t in d], np.int64))
    print("greedy done", flush=True)


def gen_native():
    """Cases: (mode, fused_ops, layer_norm, decay_mode, stack_order, carried state)."""
    from lucyrnn import LucyRNN
    from lucyrnn_conf import LucyRNNConfig
    cases = {}
    specs = []
    for mode in ["train", "infer"]:
        for ln in [True, False]:
            specs.append((f"{mode}_ln{int(ln)}", mode, True, ln, "learned", 1, False))
        specs.append((f"{mode}_unfused", mode, False, True, "learned", 1, False))
        specs.append((f"{mode}_carry", mode, True, True, "learned", 1, True))
        specs.append((f"{mode}_stack2", mode, True, True, "learned", 2, False))
    specs.append(("train_prefix", "train", True, True, "prefix_sum", 1, False))
    for name, mode, fused, ln, dmode, stack, carry in specs:
        torch.manual_seed(2024)
        cfg = LucyRNNConfig(input_dim=12, hidden_dim=16, num_layers=2, vocab_size=10,
                            kernel_impl="native", is_training=(mode == "train"), fused_ops=fused,
                            layer_norm=ln, decay_mode=dmode, stack_order=stack,
                            lambda_decay=0.05)
        m = LucyRNN(cfg)
        with torch.no_grad():
            m.output_proj.weight.normal_(0, 0.3)  # zero-init (lucyrnn.py:86) hides the encoder
            m.output_proj.bias.normal_(0, 0.1)
        x = torch.randn(2, 9 if stack == 1 else 11, 12)   # stack 2: 11 frames -> 5 steps (trim)
        hs = None
        if carry:
            h0 = [torch.randn(2, 16) * 0.5 for _ in range(2)]
            s0 = [torch.randn(2, 16) * 0.5 for _ in range(2)]
            cases[name + "/h0"] = torch.stack(h0).numpy()
            cases[name + "/s0"] = torch.stack(s0).numpy()
            hs = ([t.clone() for t in h0], [t.clone() for t in s0])
        for k, v in m.state_dict().items():
            cases[name + "/param/" + k] = v.detach().clone().numpy()
        # backward through the reference's own autograd (the native path is trainable)
        xg = x.clone().requires_grad_(True)
        logits, (h, s) = m(xg, hs)
        R = torch.randn(logits.shape, generator=torch.Generator().manual_seed(7))
        (logits * R).sum().backward()
        cases[name + "/R"] = R.numpy()
        cases[name + "/grad/x"] = xg.grad.numpy()
        for k, prm in m.named_parameters():
            if prm.grad is not None:
                cases[name + "/grad/" + k] = prm.grad.numpy()
        logits, h, s = logits.detach(), [t.detach() for t in h], [t.detach() for t in s]
        cases[name + "/x"] = x.numpy()
        cases[name + "/logits"] = logits.numpy()
        cases[name + "/h"] = torch.stack(h).numpy()
        cases[name + "/s"] = torch.stack(s).numpy()
        cases[name + "/cfg"] = np.array([mode == "train", fused, ln, dmode == "prefix_sum", stack,
                                         carry], np.int64)
        print("native", name, flush=True)
    np.savez(os.path.join(HERE, "native.npz"), **cases)


def gen_module():
    """Cases: (Din, D, V, B, T, output_proj init).  'init' keeps the reference's zero output_proj
    (lucyrnn_triton.py:108-109: logits are exactly 0, the carried states carry the check);
    'proj' draws output_proj from N(0, 0.3) after construction so the logits see every layer."""
    from lucyrnn_conf import LucyRNNConfig
    from lucyrnn_triton import LucyRNNtriton
    cases = {}
    specs = [("d64_init", 10, 64, 12, 2, 11, False), ("d64_proj", 10, 64, 12, 2, 11, True),
             ("d40_proj", 6, 40, 9, 3, 7, True)]
    for name, Din, D, V, B, T, proj in specs:
        torch.manual_seed(77)
        cfg = LucyRNNConfig(input_dim=Din, hidden_dim=D, num_layers=3, vocab_size=V,
                            kernel_impl="triton", fused_ops=True, layer_norm=False, stack_order=1)
        m = LucyRNNtriton(cfg)
        if proj:
            with torch.no_grad():
                m.output_proj.weight.normal_(0, 0.3)
                m.output_proj.bias.normal_(0, 0.1)
        for k, v in m.state_dict().items():
            cases[name + "/param/" + k] = v.detach().clone().numpy()
        # the same module in fp64 (the interpreter runs the kernel in fp64 too): the reference's
        # own fp32 rounding noise |fp32 - fp64| is the conditioning floor of the parity tests
        m64 = LucyRNNtriton(cfg).double()
        m64.load_state_dict({k: v.double() for k, v in m.state_dict().items()})
        state, state64 = None, None
        for seg in range(2):
            x = torch.randn(B, T, Din)
            with torch.no_grad():
                logits, (fh, fs) = m(x, state) if state is not None else m(x)
                l64, (h64, s64) = m64(x.double(), state64) if state64 is not None else m64(x.double())
            cases[f"{name}/seg{seg}/x"] = x.numpy()
            cases[f"{name}/seg{seg}/logits"] = logits.numpy()
            cases[f"{name}/seg{seg}/h"] = torch.stack(fh[0]).numpy()
            cases[f"{name}/seg{seg}/s"] = torch.stack(fs[0]).numpy()
            cases[f"{name}/seg{seg}/logits64"] = l64.numpy()
            cases[f"{name}/seg{seg}/h64"] = torch.stack(h64[0]).numpy()
            cases[f"{name}/seg{seg}/s64"] = torch.stack(s64[0]).numpy()
            # next segment's state: detached and contiguous (the reference kernel reads h0 as
            # contiguous memory; its strided out[:, -1] view would mis-read rows b >= 1, F3)
            state = ([[t.detach().contiguous() for t in fh[0]]], [[t.detach().clone() for t in fs[0]]])
            state64 = ([[t.detach().contiguous() for t in h64[0]]], [[t.detach().clone() for t in s64[0]]])
        print("module", name, flush=True)
    np.savez(os.path.join(HERE, "module.npz"), **cases)


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["scan", "decay", "ctc", "greedy", "native", "module"]
    for w in which:
        {"scan": gen_scan, "decay": gen_decay, "ctc": gen_ctc, "greedy": gen_greedy,
         "native": gen_native, "module": gen_module}[w]()
