"""TORCH_LIBRARY(statecatcher) registration (csrc/torch_ops.cpp + statecatcher_amd/torch_library.py)
on the CPU: the extension loads, every op has its schema, the Meta kernels give the HIP kernels'
output shapes/dtypes, the autograd formulas trace (make_fx) into the *_bwd ops, and CPU tensors
are refused (no CPU kernel, no fallback)."""
import pytest
import torch
from torch.fx.experimental.proxy_tensor import make_fx

from statecatcher_amd import _lib
from statecatcher_amd import torch_library as tl

META = torch.device("meta")


@pytest.fixture(scope="module")
def sc():
    return tl.load()


def test_every_op_registered(sc):
    for name in tl.OPS:
        assert hasattr(sc, name), name
    assert sc.abi_version() == _lib.ABI_VERSION
    s = str(torch.ops.statecatcher.lucy_scan_fwd.default._schema)
    assert "Tensor? gate_bias=None" in s and "bool need_ckpt=True" in s


@pytest.mark.parametrize("layout", ["ref", "blocked"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_scan_meta_shapes(sc, layout, dtype):
    B, T, D = 3, 100, 128
    shape = (B, T, 7, D) if layout == "ref" else (B, T, D // 64, 7, 64)
    g = torch.empty(shape, device=META, dtype=dtype)
    h = torch.empty(B, D, device=META)
    out, s, hl, ck = sc.lucy_scan_fwd(g, h, h, None, True)
    assert out.shape == (B, T, D) and out.dtype == dtype
    assert s.shape == hl.shape == (B, D) and s.dtype == hl.dtype == torch.float32
    assert ck.numel() == _lib.load().sc_lucy_scan_ckpt_numel(B, T, D)
    assert sc.lucy_scan_fwd(g, h, h, None, False)[3].numel() == 0
    dg, dh, ds, db = sc.lucy_scan_bwd(g, ck, out, None, None, True)
    assert dg.shape == g.shape and dg.dtype == dtype
    assert dh.shape == ds.shape == (B, D) and db.shape == (B, 7, D)


def test_other_meta_shapes(sc):
    kv = torch.empty(2, 9, 64, device=META, dtype=torch.bfloat16)
    assert sc.decay_scan_fwd(kv, kv, None).shape == kv.shape
    dkv, dd, di = sc.decay_scan_bwd(kv, kv, kv, torch.empty(2, 64, device=META))
    assert dkv.shape == dd.shape == kv.shape and di.shape == (2, 64)
    x = torch.empty(2, 5, 512, device=META, dtype=torch.bfloat16)
    g = torch.empty(512, device=META)
    y, mu, rs = sc.layer_norm_fwd(x, g, g, 1e-5)
    assert y.shape == x.shape and y.dtype == x.dtype and mu.shape == rs.shape == (10,)
    lg = torch.empty(4, 50, 30, device=META)
    tg = torch.empty(4, 7, device=META, dtype=torch.long)
    ln = torch.empty(4, device=META, dtype=torch.long)
    nll, ws = sc.ctc_fwd(lg, tg, ln, ln, 0, True)
    assert nll.shape == (4,) and ws.dtype == torch.uint8
    assert ws.numel() == _lib.load().sc_ctc_workspace_bytes(4, 50, 7)
    assert sc.ctc_bwd(lg, tg, ln, ln, nll, ws, nll, 0, True).shape == lg.shape
    loss, factor = sc.ctc_mean(nll, ln)
    assert loss.shape == () and factor.shape == (4,)
    tok, cnt = sc.ctc_greedy_decode(lg, ln, 0)
    assert tok.shape == (4, 50) and tok.dtype == torch.int32 and cnt.shape == (4,)


def test_meta_shape_errors(sc):
    with pytest.raises(RuntimeError, match="gates must be"):
        sc.lucy_scan_fwd(torch.empty(2, 3, 6, 8, device=META), torch.empty(2, 8, device=META),
                         torch.empty(2, 8, device=META), None, True)
    with pytest.raises(RuntimeError, match="targets must be padded"):
        sc.ctc_fwd(torch.empty(2, 5, 6, device=META), torch.empty(3, 2, device=META, dtype=torch.long),
                   torch.empty(2, device=META, dtype=torch.long),
                   torch.empty(2, device=META, dtype=torch.long), 0, True)


def _step(gates, h0, s0, bias, W, tg, il, tgl):
    out, s, h = tl.lucy_scan(gates, h0, s0, bias)
    D = out.shape[-1]
    y = tl.layer_norm(out, torch.ones(D, device=out.device), torch.zeros(D, device=out.device))
    loss = tl.ctc_loss(y.float() @ W, tg, il, tgl)
    return torch.autograd.grad(loss + h.sum() + s.sum(), (gates, h0, s0, bias, W))


def _inputs(dev):
    B, T, D, V = 2, 16, 128, 12
    mk = lambda *s, **k: torch.zeros(*s, device=dev, **k)  # noqa: E731
    return (mk(B, T, 7, D, dtype=torch.bfloat16).requires_grad_(), mk(B, D).requires_grad_(),
            mk(B, D).requires_grad_(), mk(7, D).requires_grad_(), mk(D, V).requires_grad_(),
            mk(B, 4, dtype=torch.long), torch.full((B,), T, device=dev, dtype=torch.long),
            torch.full((B,), 4, device=dev, dtype=torch.long))


def test_autograd_traces_into_backward_ops():
    """A LucyRNN layer + LayerNorm + CTC step differentiated symbolically: the graph holds the
    forward ops AND their registered backward ops (what torch.compile / AOTAutograd sees)."""
    tl.load()
    args = _inputs(META)
    grads = _step(*args)
    assert [tuple(g.shape) for g in grads] == [tuple(a.shape) for a in args[:5]]
    assert grads[0].dtype == torch.bfloat16
    gm = make_fx(_step)(*args)
    names = [str(n.target) for n in gm.graph.nodes if "statecatcher" in str(n.target)]
    for op in ("lucy_scan_fwd", "lucy_scan_bwd", "layer_norm_fwd", "layer_norm_bwd", "ctc_fwd",
               "ctc_bwd", "ctc_mean"):
        assert f"statecatcher.{op}.default" in names, (op, names)


def test_cpu_tensors_are_refused(sc):
    g = torch.zeros(1, 4, 7, 64)
    h = torch.zeros(1, 64)
    with pytest.raises(NotImplementedError):
        sc.lucy_scan_fwd(g, h, h, None, False)


def test_mlstm_and_rnnt_joint_meta_and_autograd_trace(sc):
    """The P1 ops (mlstm_*, rnnt_*): Meta shapes, and their autograd formulas trace
    into the backward ops."""
    B, NH, T, DQ, DV = 2, 4, 128, 96, 192
    q = torch.empty(B, NH, T, DQ, device=META, dtype=torch.bfloat16, requires_grad=True)
    k = torch.empty(B, NH, T, DQ, device=META, dtype=torch.bfloat16, requires_grad=True)
    v = torch.empty(B, NH, T, DV, device=META, dtype=torch.bfloat16, requires_grad=True)
    ig = torch.empty(B, NH, T, device=META, requires_grad=True)
    fg = torch.empty(B, NH, T, device=META, requires_grad=True)
    h, (c, n, m) = tl.mlstm(q, k, v, ig, fg)
    assert h.shape == (B, NH, T, DV) and h.dtype == torch.bfloat16
    assert c.shape == (B, NH, DQ, DV) and c.dtype == torch.float32
    assert n.shape == (B, NH, DQ) and m.shape == (B, NH, 1)

    def f_ml(q, k, v, ig, fg):
        h, (c, n, m) = tl.mlstm(q, k, v, ig, fg)
        return torch.autograd.grad(h.float().sum() + c.sum(), (q, k, v, ig, fg))
    gm = make_fx(f_ml)(q, k, v, ig, fg)
    names = [str(x.target) for x in gm.graph.nodes if "statecatcher" in str(x.target)]
    assert "statecatcher.mlstm_fwd.default" in names and "statecatcher.mlstm_bwd.default" in names

    T2, U, V, J = 40, 6, 64, 64
    enc = torch.empty(B, T2, J, device=META, requires_grad=True)
    pred = torch.empty(B, U + 1, J, device=META, requires_grad=True)
    W = torch.empty(V, J, device=META, requires_grad=True)
    bias = torch.empty(V, device=META, requires_grad=True)
    lab = torch.empty(B, U, device=META, dtype=torch.long)
    ln = torch.empty(B, device=META, dtype=torch.long)
    nll = tl.rnnt_joint_nll(enc, pred, W, bias, lab, ln, ln)
    assert nll.shape == (B,) and nll.dtype == torch.float32

    def f_j(enc, pred, W, bias):
        return torch.autograd.grad(tl.rnnt_joint_nll(enc, pred, W, bias, lab, ln, ln).sum(),
                                   (enc, pred, W, bias))
    gm = make_fx(f_j)(enc, pred, W, bias)
    names = [str(x.target) for x in gm.graph.nodes if "statecatcher" in str(x.target)]
    assert "statecatcher.rnnt_joint_fwd.default" in names
    assert "statecatcher.rnnt_joint_bwd.default" in names
    with pytest.raises(RuntimeError, match="multiple of 64"):
        sc.mlstm_fwd(q[:, :, :100], k[:, :, :100], v[:, :, :100], ig[:, :, :100], fg[:, :, :100])


def test_gemm_and_adam_meta(sc):
    """The projection GEMM, weight-gradient and optimizer ops: schemas and Meta shapes."""
    a = torch.empty(4096, 512, device=META, dtype=torch.bfloat16)
    w = torch.empty(3584, 512, device=META, dtype=torch.bfloat16)
    c = sc.gemm_tn(a, w, 0)
    assert c.shape == (4096, 3584) and c.dtype == torch.bfloat16
    dy = torch.empty(4096, 3584, device=META, dtype=torch.bfloat16)
    dw = sc.gemm_wgrad(dy, a, 512)
    assert dw.shape == (3584, 512) and dw.dtype == torch.float32
    p = [torch.empty(10, device=META), torch.empty(3, 4, device=META)]
    n = sc.clip_adam_(p, p, p, p, 1, 50.0, 1e-3, 0.9, 0.999, 1e-8, 0.0, False, 1e-3, 0.03)
    assert n.shape == () and n.dtype == torch.float32
    s = str(torch.ops.statecatcher.clip_adam_.default._schema)
    assert "Tensor(a!)[] params" in s and "Tensor(b!)[] exp_avgs" in s


def test_gemm_ops_refuse_cpu(sc):
    a = torch.zeros(256, 64, dtype=torch.bfloat16)
    with pytest.raises((RuntimeError, NotImplementedError)):
        sc.gemm_tn(a, a, 0)
    with pytest.raises((RuntimeError, NotImplementedError)):
        sc.gemm_wgrad(a, a, 0)
