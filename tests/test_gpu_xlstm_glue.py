"""GPU parity of the fused xLSTM block glue (csrc/xlstm_glue.hip) against the torch modules' own
computation under bf16 autocast (statecatcher_amd/xlstm.py's torch path, the restatement of
transformers' modeling_xlstm.py RMSNorm / MultiHeadLayerNorm / FFN).

The fused kernels round to bf16 at the same points as the torch chain, so outputs agree to a
bf16 ulp (2^-8 of the value, from reduction order); gradients to 2e-2 in norm (the torch
backward rounds some intermediates to bf16 that the kernels keep in fp32) and weight gradients
(fp32 sums over all rows) to 1e-2 in norm."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def ops():
    from statecatcher_amd import ops as o
    return o


def rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


def ulp_close(a, b):
    err = (a.float() - b.float()).abs()
    return bool((err <= b.float().abs() * 2.0 ** -7 + 1e-3 * b.float().abs().max()).all())


@pytest.mark.parametrize("D,rows", [(768, 4000), (512, 33), (1024, 7)])
def test_rmsnorm_vs_torch(D, rows):
    g = torch.Generator(device=DEV).manual_seed(D + rows)
    x = (torch.randn(rows, D, device=DEV, generator=g) * 2).to(torch.bfloat16)
    w = (1 + 0.3 * torch.randn(D, device=DEV, generator=g))
    dy = torch.randn(rows, D, device=DEV, generator=g).to(torch.bfloat16)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = ((xr.float() * torch.rsqrt(xr.float().pow(2).mean(-1, keepdim=True) + 1e-6)).to(torch.bfloat16)
          * wr).to(torch.bfloat16)
    yr.backward(dy)
    xf = x.clone().requires_grad_(True)
    wf = w.clone().requires_grad_(True)
    yf = ops().rms_norm(xf, wf, 1e-6)
    yf.backward(dy)
    assert yf.dtype == torch.bfloat16 and ulp_close(yf, yr)
    assert rel(xf.grad, xr.grad) < 2e-2
    assert rel(wf.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("B,NH,T,DH", [(2, 4, 65, 192), (3, 2, 9, 64), (1, 4, 128, 256)])
def test_gated_head_norm_vs_torch(B, NH, T, DH):
    g = torch.Generator(device=DEV).manual_seed(B * T + DH)
    h = (torch.randn(B, NH, T, DH, device=DEV, generator=g) * 3 + 0.5).to(torch.bfloat16)
    proj = torch.randn(B, T, NH * DH + 40, device=DEV, generator=g).to(torch.bfloat16)
    o = proj[..., 8:8 + NH * DH]                     # a row-strided view, as in the layer
    w = 1 + 0.3 * torch.randn(NH * DH, device=DEV, generator=g)
    dy = torch.randn(B, T, NH * DH, device=DEV, generator=g).to(torch.bfloat16)
    hr, orr, wr = (t.clone().requires_grad_(True) for t in (h, o, w))
    y = hr.transpose(1, 2).float()
    y = (y - y.mean(-1, keepdim=True)) * torch.rsqrt(y.var(-1, keepdim=True, unbiased=False) + 1e-6)
    y = y.to(torch.bfloat16).reshape(B, T, -1) * wr
    outr = (torch.sigmoid(orr) * y).to(torch.bfloat16)
    outr.backward(dy)
    hf, of, wf = (t.clone().requires_grad_(True) for t in (h, o, w))
    outf = ops().gated_head_norm(hf, of, wf, 1e-6)
    outf.backward(dy)
    assert outf.shape == outr.shape and ulp_close(outf, outr)
    assert rel(hf.grad, hr.grad) < 2e-2
    assert rel(of.grad, orr.grad) < 2e-2
    assert rel(wf.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("rows,Fd", [(3000, 2048), (5, 64)])
def test_swiglu_vs_torch(rows, Fd):
    g = torch.Generator(device=DEV).manual_seed(rows)
    a = (torch.randn(rows, 2 * Fd, device=DEV, generator=g) * 2).to(torch.bfloat16)
    dy = torch.randn(rows, Fd, device=DEV, generator=g).to(torch.bfloat16)
    ar = a.clone().requires_grad_(True)
    gr, ur = ar.split([Fd, Fd], -1)
    yr = F.silu(gr) * ur
    yr.backward(dy)
    af = a.clone().requires_grad_(True)
    yf = ops().swiglu(af)
    yf.backward(dy)
    assert ulp_close(yf, yr)
    assert rel(af.grad, ar.grad) < 2e-2


@pytest.mark.parametrize("D,rows", [(768, 3000), (512, 5)])
def test_add_rms_norm_bitwise_vs_add_then_norm(D, rows):
    """AddRMSNormFn (residual add folded into the RMSNorm, the residual gradient folded into its
    backward) against x + r followed by RMSNormFn: the same bf16 roundings, so the sum, the
    normalised output and every gradient are bitwise equal."""
    g = torch.Generator(device=DEV).manual_seed(D * rows)
    x = (torch.randn(rows, D, device=DEV, generator=g) * 2).to(torch.bfloat16)
    r = torch.randn(rows, D, device=DEV, generator=g).to(torch.bfloat16)
    w = 1 + 0.3 * torch.randn(D, device=DEV, generator=g)
    ds = torch.randn(rows, D, device=DEV, generator=g).to(torch.bfloat16)
    dn = torch.randn(rows, D, device=DEV, generator=g).to(torch.bfloat16)
    res = []
    for fused in (True, False):
        xi, ri, wi = (t.clone().requires_grad_(True) for t in (x, r, w))
        if fused:
            sm, n = ops().add_rms_norm(xi, ri, wi, 1e-6)
        else:
            sm = xi + ri
            n = ops().rms_norm(sm, wi, 1e-6)
        torch.autograd.backward((sm, n), (ds, dn))
        res.append((sm.detach(), n.detach(), xi.grad, ri.grad, wi.grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_xlstm_unrolled_model_equals_block_loop():
    """xLSTMLarge.forward (every residual add folded into the next RMSNorm) against the plain
    loop over xLSTMBlock.forward with the inter-block adds as torch adds: bitwise equal logits
    and parameter gradients under bf16 autocast."""
    from statecatcher_amd import xlstm
    cfg = xlstm.xLSTMLargeConfig(embedding_dim=256, num_heads=4, num_blocks=2, vocab_size=64,
                                 input_dim=80)
    torch.manual_seed(1)
    model = xlstm.xLSTMLarge(cfg).to(DEV)
    feats = torch.randn(2, 128, 80, device=DEV)

    def loop(x):
        x = model.embedding(x)
        for blk in model.blocks:
            x, _ = blk(x)
        return xlstm.soft_cap(model.lm_head(model.out_norm(x)), cfg.output_logit_soft_cap)

    res = []
    for fn in (lambda f: model(f)[0], loop):
        model.zero_grad()
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits = fn(feats)
        logits.float().square().mean().backward()
        res.append((logits.detach(), {n: p.grad.clone() for n, p in model.named_parameters()}))
    (la, ga), (lb, gb) = res
    assert torch.equal(la, lb)
    for n in ga:
        assert torch.equal(ga[n], gb[n]), n


def test_xlstm_block_fused_equals_torch_path():
    """A whole xLSTM block under bf16 autocast: fused glue vs the torch path (glue disabled)."""
    from statecatcher_amd import xlstm
    cfg = xlstm.xLSTMLargeConfig(embedding_dim=256, num_heads=4, num_blocks=1, vocab_size=64)
    torch.manual_seed(0)
    blk = xlstm.xLSTMBlock(cfg).to(DEV)
    x = torch.randn(2, 128, 256, device=DEV)
    outs = []
    for fused in (True, False):
        saved = (xlstm.ops.xlstm_glue_supported, xlstm.ops.gated_head_norm_supported,
                 xlstm.ops.mlstm_core_supported)
        if not fused:
            xlstm.ops.xlstm_glue_supported = lambda *a: False
            xlstm.ops.gated_head_norm_supported = lambda *a: False
            xlstm.ops.mlstm_core_supported = lambda *a: False
        try:
            blk.zero_grad()
            xi = x.clone().requires_grad_(True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y, _ = blk(xi.to(torch.bfloat16))
            y.float().square().mean().backward()
            outs.append((y.float(), xi.grad.clone(),
                         {n: p.grad.clone() for n, p in blk.named_parameters()}))
        finally:
            (xlstm.ops.xlstm_glue_supported, xlstm.ops.gated_head_norm_supported,
             xlstm.ops.mlstm_core_supported) = saved
    (yf, gxf, pf), (yt, gxt, pt) = outs
    assert rel(yf, yt) < 1e-2
    assert rel(gxf, gxt) < 3e-2
    # per parameter, with a floor at 1e-3 of the largest gradient: the gate biases' gradients
    # (~1e-6 here, 1e5 below the others) are rounding noise in both paths
    gmax = max(float(t.norm()) for t in pt.values())
    for n in pt:
        err = float((pf[n].double() - pt[n].double()).norm())
        assert err <= 3e-2 * float(pt[n].norm()) + 1e-3 * gmax, (n, err, float(pt[n].norm()))


@pytest.mark.parametrize("kernel_dtype", ["bfloat16", "float16"])
@pytest.mark.parametrize("with_state", [False, True])
def test_mlstm_core_equals_composed_ops(with_state, kernel_dtype, monkeypatch):
    """ops.MLSTMCoreFn (q/k/v/o read in place from the fused projection, one gradient tensor
    written in place) against the composed path it replaces (split, soft caps, MLSTMFn,
    GatedHeadNormFn, autograd's concatenation): the layer output and the final state are
    bit-identical; the gradients agree to 1e-2 (relative Frobenius; measured ~1e-3): the core
    path takes the gate gradients through the soft cap in fp32 with one bf16 rounding
    (sc_mlstm_gate_bwd), the composed path through torch's five bf16 ops.  With the reference's
    float16 cell the
    core path reads the bf16 projection and rounds to f16 on load (sc_mlstm_*_io) where the split
    path casts: the forward is still bit-identical; in the backward the split path also casts
    the bf16 dh to f16, which is exact only in f16's normal range, while the core path reads dh
    as bf16 -- so there the gradients agree to 1e-2 (relative Frobenius, with the loss scaled so
    that most of dh is in f16's normal range; the |dh| < 6e-5 elements differ) and the core
    path's are the more accurate (unscaled, the split path's f16 dh costs 7% on q.weight)."""
    from statecatcher_amd import xlstm
    cfg = xlstm.xLSTMLargeConfig(embedding_dim=256, num_heads=4, num_blocks=1, vocab_size=64,
                                 autocast_kernel_dtype=kernel_dtype)
    torch.manual_seed(1)
    layer = xlstm.mLSTMLayer(cfg).to(DEV)
    with torch.no_grad():
        for m in layer._mods():
            m.weight.mul_(3.0)
        layer.multihead_norm.weight.uniform_(0.5, 1.5)
    x = torch.randn(2, 192, 256, device=DEV)
    st = None
    if with_state:
        g = torch.Generator(device=DEV).manual_seed(2)
        st = (torch.randn(2, 4, 32, 64, device=DEV, generator=g) * 0.1,
              torch.randn(2, 4, 32, device=DEV, generator=g) * 0.1,
              torch.zeros(2, 4, 1, device=DEV))
    res = []
    for core in (True, False):
        if not core:
            monkeypatch.setattr(xlstm.ops, "mlstm_core_supported", lambda *a: False)
        layer.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(True)
        sti = None if st is None else tuple(t.clone().requires_grad_(i < 2) for i, t in enumerate(st))
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y, (c, n, m) = layer(xi, sti)
        # (scaled: dh mostly inside f16's normal range, see above)
        (4096.0 * y.float().square().mean() + c.square().mean() + n.mean()).backward()
        res.append([y, c, n, m, xi.grad] + [p.grad for p in layer.parameters()] +
                   ([sti[0].grad, sti[1].grad] if sti else []))
    for i, (u, v) in enumerate(zip(*res)):
        if i < 4:
            assert torch.equal(u, v), i
        else:
            rel = float((u.double() - v.double()).norm() / max(float(v.double().norm()), 1e-30))
            assert rel <= 1e-2, (i, rel)


def test_fused_linear_bitwise_vs_cat_then_linear():
    """FusedLinearFn (bf16 image of the row-concatenated weights in one sc_weight_images launch,
    weight gradient split back per weight) against torch.cat -> AutocastLinearFn: the same
    roundings, so output and every gradient are bitwise equal."""
    g = torch.Generator(device=DEV).manual_seed(21)
    x = torch.randn(3, 640, 768, device=DEV, generator=g).to(torch.bfloat16)
    ws = [torch.randn(n, 768, device=DEV, generator=g) * 0.02 for n in (384, 384, 768, 768, 4, 4)]
    b = torch.cat([torch.zeros(2304, device=DEV), torch.randn(8, device=DEV, generator=g)])
    dy = torch.randn(3, 640, 2312, device=DEV, generator=g).to(torch.bfloat16)
    res = []
    for fused in (True, False):
        xi = x.clone().requires_grad_(True)
        wi = [w.clone().requires_grad_(True) for w in ws]
        bi = b.clone().requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert ops().fused_linear_ok(xi, wi)
            y = (ops().fused_linear(xi, wi, bi, 2304) if fused
                 else ops().autocast_linear(xi, torch.cat(wi), bi, 2304))
        y.backward(dy)
        res.append([y.detach(), xi.grad, bi.grad] + [w.grad for w in wi])
    for a, c in zip(*res):
        assert torch.equal(a, c)


@pytest.mark.parametrize("cap", [15.0, None])
def test_mlstm_gate_bwd_kernel_vs_torch_chain(cap):
    """sc_mlstm_gate_bwd against what it replaced in MLSTMFn / MLSTMCoreFn: d fgate =
    sigmoid(-f) * flip(cumsum(flip(qdq - kdk))) in fp32 (the kernel's suffix sums run in another
    order: 1e-5 relative), and the soft-cap backward: against fp64 g (1 - tanh(x / cap)^2) to
    one bf16 rounding, and at least as close to it as the torch chain (ops._soft_cap_bwd, five
    bf16 roundings).  Columns outside the two gate groups are untouched."""
    from statecatcher_amd import _lib
    from statecatcher_amd.ops import _soft_cap_bwd, ptr
    g = torch.Generator(device=DEV).manual_seed(4)
    B, NH, T = 3, 4, 384
    io, fo, N = 8, 20, 40
    qdq = torch.randn(B * NH, T, device=DEV, generator=g)
    kdk = torch.randn(B * NH, T, device=DEV, generator=g) * 0.5
    fg = torch.randn(B * NH, T, device=DEV, generator=g) * 3 + 2
    a = (torch.randn(B, T, N, device=DEV, generator=g) * 20).to(torch.bfloat16)
    lib = _lib.load()
    dfg = torch.empty_like(kdk)
    assert lib.sc_mlstm_gate_bwd(ptr(qdq), ptr(kdk), ptr(fg), B * NH, T, ptr(dfg), None, None, 0, 0,
                                 0, 0, 0.0, None) == 0
    da = torch.zeros_like(a)
    assert lib.sc_mlstm_gate_bwd(ptr(qdq), ptr(kdk), ptr(fg), B * NH, T, None, ptr(a), ptr(da), NH,
                                 N, io, fo, cap or 0.0, None) == 0
    torch.cuda.synchronize()
    ref_dfg = torch.sigmoid(-fg) * (qdq - kdk).flip(-1).cumsum(-1).flip(-1)
    torch.testing.assert_close(dfg, ref_dfg, rtol=1e-5, atol=1e-5 * float(ref_dfg.abs().max()))
    for col, gr in ((io, kdk), (fo, dfg)):
        gt = gr.view(B, NH, T).transpose(1, 2).double()
        x = a[..., col:col + NH].double()
        exact = gt if cap is None else gt * (1 - torch.tanh(x / cap) ** 2)
        got = da[..., col:col + NH].double()
        err = (got - exact).abs()
        assert bool((err <= 2.0 ** -8 * exact.abs() + 1e-30).all())
        chain = _soft_cap_bwd(gt.to(torch.bfloat16), a[..., col:col + NH], cap).double()
        assert float(err.norm()) <= float((chain - exact).norm()) + 1e-30
    assert not da[..., :io].any() and not da[..., io + NH:fo].any() and not da[..., fo + NH:].any()
