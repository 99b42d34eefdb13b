"""GPU parity of the TORCH_LIBRARY(statecatcher) ops (csrc/torch_ops.cpp): the dispatcher path
launches the same kernels as the ctypes autograd nodes of ops.py, so results are compared
BITWISE against them (and the scan against the oracle, tolerances as test_gpu_scan.py);
torch.library.opcheck validates schema / fake / autograd registration; torch.compile with
fullgraph=True runs the ops without graph breaks and matches eager."""
import numpy as np
import pytest
import torch

from oracle import ctc as octc
from oracle import lucy_scan as oscan

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _tl():
    from statecatcher_amd import torch_library as tl
    tl.load()
    return tl


def _ops():
    from statecatcher_amd import ops
    return ops


def _scan_inputs(B, T, D, dtype, seed=0):
    g = torch.Generator().manual_seed(seed)
    gates = (torch.randn(B, T, 7, D, generator=g) * 0.5).to(DEV, dtype)
    h0 = (torch.randn(B, D, generator=g) * 0.1).to(DEV)
    s0 = (torch.randn(B, D, generator=g) * 0.1).to(DEV)
    dout = torch.randn(B, T, D, generator=g).to(DEV, dtype)
    return gates, h0, s0, dout


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 130, 96), (3, 257, 128), (1, 64, 512)])
def test_scan_bitwise_vs_ctypes_path_and_oracle(shape, dtype):
    tl, ops = _tl(), _ops()
    gates, h0, s0, dout = _scan_inputs(*shape, dtype)
    g1 = gates.clone().requires_grad_()
    out1, s1, hl1 = tl.lucy_scan(g1, h0, s0)
    (out1.float() * dout.float()).sum().backward()
    g2 = gates.clone().requires_grad_()
    out2, s2 = ops.lucy_scan(g2, h0, s0)
    (out2.float() * dout.float()).sum().backward()
    torch.cuda.synchronize()
    assert torch.equal(out1, out2) and torch.equal(s1, s2)
    assert torch.equal(g1.grad, g2.grad)
    if dtype == torch.float32:
        ref_out, ref_s = oscan.lucy_scan_fwd(gates.cpu().numpy(), h0.cpu().numpy(), s0.cpu().numpy())
        np.testing.assert_allclose(out1.detach().cpu().numpy(), ref_out, rtol=1e-3, atol=1e-5)
        np.testing.assert_allclose(hl1.detach().cpu().numpy(), ref_out[:, -1], rtol=1e-3, atol=1e-5)
        np.testing.assert_allclose(s1.detach().cpu().numpy(), ref_s, rtol=1e-3, atol=1e-5)


def test_scan_state_and_bias_gradients_vs_oracle():
    """dh0/ds0 and the gate-bias gradient (bias added on load) against the fp32 oracle."""
    tl = _tl()
    B, T, D = 2, 200, 128
    gates, h0, s0, dout = _scan_inputs(B, T, D, torch.float32, seed=3)
    bias = (torch.randn(7, D, generator=torch.Generator().manual_seed(4)) * 0.2).to(DEV)
    gq, hq, sq, bq = (t.clone().requires_grad_() for t in (gates, h0, s0, bias))
    out, s_last, _ = tl.lucy_scan(gq, hq, sq, bq)
    (out * dout).sum().backward()
    gb = (gates + bias.view(1, 1, 7, D)).cpu().numpy()
    ref_dg, ref_dh0, ref_ds0 = oscan.lucy_scan_bwd(gb, h0.cpu().numpy(), s0.cpu().numpy(),
                                                   dout.cpu().numpy(), np.zeros((B, D), np.float32))
    for got, ref in ((gq.grad, ref_dg), (hq.grad, ref_dh0), (sq.grad, ref_ds0),
                     (bq.grad, ref_dg.sum(axis=(0, 1)))):
        sc = max(np.abs(ref).max(), 1e-6)
        np.testing.assert_allclose(got.cpu().numpy(), ref, rtol=1e-3, atol=1e-3 * sc)


def test_ctc_loss_bitwise_vs_ctypes_path_and_oracle():
    tl, ops = _tl(), _ops()
    g = torch.Generator().manual_seed(1)
    B, T, V, U = 4, 120, 40, 30
    logits = torch.randn(B, T, V, generator=g).to(DEV)
    tg = torch.randint(1, V, (B, U), generator=g).to(DEV)
    il = torch.tensor([120, 100, 90, 20], device=DEV)   # the last is infeasible: zero_infinity
    tgl = torch.tensor([30, 25, 1, 30], device=DEV)
    x1 = logits.clone().requires_grad_()
    l1 = tl.ctc_loss(x1, tg, il, tgl)
    l1.backward()
    x2 = logits.clone().requires_grad_()
    l2 = ops.ctc_loss(x2, tg, il, tgl)
    l2.backward()
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(x1.grad, x2.grad)
    rn, _ = octc.ctc_loss_grad(logits[:3].cpu().numpy(), tg[:3].cpu().numpy(), il[:3].tolist(),
                               tgl[:3].tolist())
    nll = tl.ctc_nll(logits, tg, il, tgl).cpu().numpy()
    np.testing.assert_allclose(nll[:3], rn[:3], rtol=1e-4)
    assert np.isinf(nll[3])


def test_decay_scan_layer_norm_greedy_bitwise():
    tl, ops = _tl(), _ops()
    g = torch.Generator().manual_seed(2)
    kv = torch.randn(2, 300, 128, generator=g).to(DEV)
    dec = torch.rand(2, 300, 128, generator=g).to(DEV)
    init = torch.randn(2, 128, generator=g).to(DEV)
    a = [t.clone().requires_grad_() for t in (kv, dec, init)]
    b = [t.clone().requires_grad_() for t in (kv, dec, init)]
    ya, yb = tl.decay_scan(*a), ops.decay_scan(*b)
    ya.sum().backward()
    yb.sum().backward()
    assert torch.equal(ya, yb)
    for p, q in zip(a, b):
        assert torch.equal(p.grad, q.grad)
    x = torch.randn(3, 50, 512, generator=g).to(DEV, torch.bfloat16)
    gm = torch.randn(512, generator=g).to(DEV)
    bt = torch.randn(512, generator=g).to(DEV)
    xa, ga, ba = (t.clone().requires_grad_() for t in (x, gm, bt))
    xb, gb, bb = (t.clone().requires_grad_() for t in (x, gm, bt))
    dy = torch.randn(3, 50, 512, generator=g).to(DEV, torch.bfloat16)
    (tl.layer_norm(xa, ga, ba).float() * dy.float()).sum().backward()
    (ops.layer_norm(xb, gb, bb).float() * dy.float()).sum().backward()
    for p, q in ((xa, xb), (ga, gb), (ba, bb)):
        assert torch.equal(p.grad, q.grad)
    lp = torch.randn(3, 40, 20, generator=g).to(DEV).log_softmax(-1)
    lens = torch.tensor([40, 33, 0], device=DEV)
    t1, c1 = tl.ctc_greedy_decode(lp, lens)
    t2, c2 = ops.ctc_greedy_decode(lp, lens)
    assert torch.equal(c1, c2)
    for b in range(3):
        assert torch.equal(t1[b, :c1[b]], t2[b, :c2[b]])


def test_opcheck():
    """Schema, fake (Meta) kernels vs real outputs, and autograd registration."""
    tl = _tl()
    sc = torch.ops.statecatcher
    gates, h0, s0, _ = _scan_inputs(2, 70, 64, torch.float32)
    torch.library.opcheck(sc.lucy_scan_fwd.default, (gates.requires_grad_(), h0, s0, None, True),
                          test_utils=("test_schema", "test_faketensor",
                                      "test_autograd_registration"))
    kv = torch.randn(2, 33, 64, device=DEV)
    torch.library.opcheck(sc.decay_scan_fwd.default, (kv.requires_grad_(), torch.rand_like(kv), None),
                          test_utils=("test_schema", "test_faketensor",
                                      "test_autograd_registration"))
    x = torch.randn(4, 512, device=DEV, requires_grad=True)
    w = torch.ones(512, device=DEV)
    torch.library.opcheck(sc.layer_norm_fwd.default, (x, w, torch.zeros_like(w), 1e-5),
                          test_utils=("test_schema", "test_faketensor",
                                      "test_autograd_registration"))
    lg = torch.randn(2, 30, 9, device=DEV, requires_grad=True)
    tg = torch.randint(1, 9, (2, 5), device=DEV)
    ln = torch.tensor([30, 28], device=DEV)
    tln = torch.tensor([5, 3], device=DEV)
    torch.library.opcheck(sc.ctc_fwd.default, (lg, tg, ln, tln, 0, True),
                          test_utils=("test_schema", "test_faketensor",
                                      "test_autograd_registration"))
    assert tl is not None


def test_torch_compile_fullgraph_matches_eager():
    """A LucyRNN layer (scan + LayerNorm) + CTC loss under torch.compile(fullgraph=True): no graph
    break at the custom ops, same loss and gradients as eager (the same kernels run)."""
    tl = _tl()
    B, T, D, V, U = 2, 96, 256, 16, 10   # fp32 LayerNorm: D in 256 * {1, 2, 4, 8}
    g = torch.Generator().manual_seed(5)
    gates = (torch.randn(B, T, 7, D, generator=g) * 0.5).to(DEV)
    W = (torch.randn(D, V, generator=g) * 0.1).to(DEV)
    tg = torch.randint(1, V, (B, U), generator=g).to(DEV)
    il = torch.full((B,), T, device=DEV)
    tgl = torch.tensor([U, U - 3], device=DEV)
    zero = torch.zeros(B, D, device=DEV)
    gamma = torch.ones(D, device=DEV)
    beta = torch.zeros(D, device=DEV)

    def f(gates, W):
        out, _, _ = tl.lucy_scan(gates, zero, zero)
        y = tl.layer_norm(out, gamma, beta)
        return tl.ctc_loss(y @ W, tg, il, tgl)

    def run(fn):
        gq, wq = gates.clone().requires_grad_(), W.clone().requires_grad_()
        loss = fn(gq, wq)
        loss.backward()
        return loss.detach(), gq.grad, wq.grad

    torch._dynamo.reset()
    eager = run(f)
    compiled = run(torch.compile(f, fullgraph=True, backend="aot_eager"))
    for a, b in zip(eager, compiled):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_mlstm_op_bitwise_vs_ctypes_path_and_opcheck():
    """torch.ops.statecatcher.mlstm_fwd / _bwd launch the walk kernels the ctypes node
    (ops.MLSTMFn) launches: h, the final state and every gradient bitwise equal."""
    tl, ops = _tl(), _ops()
    g = torch.Generator().manual_seed(3)
    B, NH, T, DQ, DV = 2, 2, 192, 64, 128
    q, k = (torch.randn(B, NH, T, DQ, generator=g).to(DEV, torch.bfloat16) for _ in range(2))
    v = torch.randn(B, NH, T, DV, generator=g).to(DEV, torch.bfloat16)
    ig = (torch.randn(B, NH, T, generator=g) * 3).to(DEV)
    fg = (torch.randn(B, NH, T, generator=g) * 2 + 3).to(DEV)
    c0 = (torch.randn(B, NH, DQ, DV, generator=g) * 0.3).to(DEV)
    n0 = (torch.randn(B, NH, DQ, generator=g) * 0.3).to(DEV)
    R = torch.randn(B, NH, T, DV, generator=g).to(DEV)
    outs = []
    for fn in (lambda *a: tl.mlstm(*a), lambda *a: ops.mlstm_chunkwise(*a, return_last_states=True)):
        leaves = [t.clone().requires_grad_() for t in (q, k, v, ig, fg, c0, n0)]
        h, (c, n, m) = fn(*leaves)
        ((h.float() * R).sum() + c.sum() + n.sum()).backward()
        outs.append([h, c, n, m] + [t.grad for t in leaves])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    torch.library.opcheck(torch.ops.statecatcher.mlstm_fwd.default,
                          (q, k, v, ig, fg, c0, n0, None, 1e-6),
                          test_utils=("test_schema", "test_faketensor"))


def test_rnnt_joint_op_bitwise_vs_ctypes_path():
    tl, ops = _tl(), _ops()
    g = torch.Generator().manual_seed(4)
    B, T, U, V, J = 2, 37, 7, 96, 64
    enc = torch.randn(B, T, J, generator=g).to(DEV)
    pred = torch.randn(B, U + 1, J, generator=g).to(DEV)
    W = (torch.randn(V, J, generator=g) * 0.3).to(DEV)
    bias = torch.randn(V, generator=g).to(DEV)
    lab = torch.randint(1, V, (B, U), generator=g).to(DEV)
    fl = torch.tensor([T, 20], device=DEV)
    ll = torch.tensor([U, 3], device=DEV)
    outs = []
    for fn in (lambda *a: tl.rnnt_joint_nll(*a, lab, fl, ll, 0),
               lambda *a: ops.RNNTJointFn.apply(*a, lab, fl, ll, 0)):
        leaves = [t.clone().requires_grad_() for t in (enc, pred, W, bias)]
        nll = fn(*leaves)
        nll.mean().backward()
        outs.append([nll] + [t.grad for t in leaves])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_gemm_and_adam_ops_bitwise_vs_ctypes_path():
    """torch.ops.statecatcher.gemm_tn / gemm_wgrad / clip_adam_ run the same kernels as the
    ctypes nodes (ops.gemm_tn, ops.wgrad_mfma, optim.clip_and_adam_step): bitwise equal."""
    from statecatcher_amd import ops, optim
    tl = _tl()
    g = torch.Generator(device=DEV).manual_seed(3)
    M, K, N = 8192, 512, 3584
    a = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV, generator=g).to(torch.bfloat16)
    assert torch.equal(tl.gemm_tn(a, w), ops.gemm_tn(a, w))
    dy = torch.randn(M, N, device=DEV, generator=g).to(torch.bfloat16)
    for bd in (0, 512):
        assert torch.equal(tl.gemm_wgrad(dy, a, bd), ops.wgrad_mfma(dy, a, bd))
    # one clipped Adam step on two parameters against the optimizer path
    ps = [torch.randn(1000, device=DEV, generator=g), torch.randn(37, 5, device=DEV, generator=g)]
    gs = [torch.randn_like(p) * 40 for p in ps]
    q = [p.clone().requires_grad_(True) for p in ps]
    for x, gr in zip(q, gs):
        x.grad = gr.clone()
    opt = torch.optim.Adam(q, lr=1e-3)
    norm_ref = optim.clip_and_adam_step(opt, q, 50.0)
    m = [torch.zeros_like(p) for p in ps]
    v = [torch.zeros_like(p) for p in ps]
    pc = [p.clone() for p in ps]
    norm = tl.clip_adam_(pc, gs, m, v, 2, 50.0, 1e-3, (0.9, 0.999), 1e-8, 0.0, False, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(norm.reshape(()), norm_ref.reshape(()))
    for x, y, mm, vv in zip(pc, q, m, v):
        assert torch.equal(x, y.detach())
        assert torch.equal(mm, opt.state[y]["exp_avg"]) and torch.equal(vv, opt.state[y]["exp_avg_sq"])
