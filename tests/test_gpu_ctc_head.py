"""The fused output projection + CTC node (ops.CTCHeadFn) that compute_loss uses under bf16
autocast: output_proj (lucyrnn_triton.py:107-109, :150) and the lattice (model.py:68-71,
train.py:142: log_softmax + nn.CTCLoss(mean, zero_infinity)) with the lattice's emission logits at
fp32 accuracy (fp32 logits without the scan's split planes; with them, by default, bf16 logits plus
the emission columns as a side array), and the gradient to the projection backward in bf16.

* Against the same computation unfused on the same bf16 operands (fp32 logits from the bf16
  GEMM, the fp32 HIP lattice, the projection's backward in fp32 torch): loss 1e-5 relative,
  gradients 1e-2 in norm (the fused backward's bf16 dlogits and bf16 GEMMs).
* The returned logits stay differentiable: a second loss on them adds its gradient.
* compute_loss takes it exactly under bf16 autocast with CTCLoss(fused_head=True).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def sc():
    import statecatcher_amd as s
    return s


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def inputs(B=3, T=200, D=256, V=512, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(B, T, D, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    w = (torch.randn(V, D, generator=g) * 0.05).to(DEV)
    b = (torch.randn(V, generator=g) * 0.1).to(DEV)
    U = [20, 35, 0]
    tg = torch.randint(1, V, (B, 35), generator=g)
    for i, u in enumerate(U):
        tg[i, u:] = 0
    return x, w, b, tg.to(DEV), [T, T - 30, T - 7], U


def test_ctc_head_vs_unfused():
    x, w, b, tg, il, tl = inputs()
    ops = sc().ops
    wc, wt = w.to(torch.bfloat16), w.t().contiguous().to(torch.bfloat16)
    x1 = x.clone().requires_grad_(True)
    w1, b1 = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    loss, logits = ops.ctc_head_loss(x1, w1, b1, (wc, wt), tg, il, tl)
    assert logits.dtype == torch.float32
    loss.backward()
    # unfused: fp32 logits of the same bf16 operands; w, b enter through an identity-gradient
    # rounding so their gradients are d loss / d (bf16 W) as the fused node's are
    x2 = x.float().requires_grad_(True)
    w2, b2 = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    wq = w2 + (wc.float() - w2).detach()
    ref_logits = x2 @ wq.t() + b2
    ref = sc().ctc_loss(ref_logits, tg, il, tl)
    ref.backward()
    print(f"head: loss {loss.item():.6f} vs {ref.item():.6f}; logits {rel(logits, ref_logits):.1e}; "
          f"dx {rel(x1.grad, x2.grad):.2e} dW {rel(w1.grad, w2.grad):.2e} db {rel(b1.grad, b2.grad):.2e}")
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-5)
    assert rel(logits, ref_logits) < 1e-5
    for got, want in ((x1.grad, x2.grad), (w1.grad, w2.grad), (b1.grad, b2.grad)):
        assert got.dtype == want.dtype or got.dtype == torch.bfloat16
        assert rel(got, want) < 1e-2


def test_ctc_head_logits_stay_differentiable():
    x, w, b, tg, il, tl = inputs(seed=1)
    wc, wt = w.to(torch.bfloat16), w.t().contiguous().to(torch.bfloat16)
    w1 = w.clone().requires_grad_(True)
    loss, logits = sc().ops.ctc_head_loss(x, w1, b, (wc, wt), tg, il, tl)
    (loss + logits.square().sum()).backward()
    g_both = w1.grad.clone()
    w1.grad = None
    loss, logits = sc().ops.ctc_head_loss(x, w1, b, (wc, wt), tg, il, tl)
    loss.backward()
    g_ctc = w1.grad.clone()
    extra = 2.0 * (logits.detach().reshape(-1, w.shape[0]).t() @ x.float().reshape(-1, x.shape[2]))
    assert rel(g_both - g_ctc, extra) < 2e-2


def test_compute_loss_uses_head_under_bf16_autocast(monkeypatch):
    import statecatcher_amd.model as m
    calls = []
    orig = m.ctc_head_loss
    monkeypatch.setattr(m, "ctc_head_loss", lambda *a, **k: calls.append(1) or orig(*a, **k))
    cfg = sc().build_lucyrnn_config(80, 128, 2, 256)
    model = sc().ASRModel(None, cfg, vocab_size=256, feat_dim=80, proj_dim=-1).to(DEV)
    with torch.no_grad():
        model.encoder.output_proj.weight.normal_(0, 0.05)
    feats = torch.randn(2, 64, 80, device=DEV)
    masks = torch.ones(2, 64, dtype=torch.bool, device=DEV)
    tok = torch.randint(1, 256, (2, 10), device=DEV)
    crit = sc().CTCLoss(blank=0, zero_infinity=True, fused_head=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss, _, enc_out, _ = sc().compute_loss("ctc", crit, model, feats, masks, tok, [64, 64],
                                                [10, 10], 0)
    # (the split planes are present here: "emis" keeps the bf16 GEMM's logits)
    want = torch.bfloat16 if sc().ops.HEAD_SPLIT == "emis" else torch.float32
    assert calls and enc_out.dtype == want and enc_out.shape == (2, 64, 256)
    loss.backward()
    assert model.encoder.output_proj.weight.grad is not None
    # fp32 training and a non-fusing criterion keep the module's own logits
    calls.clear()
    loss, _, enc_out, _ = sc().compute_loss("ctc", crit, model, feats, masks, tok, [64, 64], [10, 10], 0)
    assert not calls and enc_out.dtype == torch.float32
    with torch.autocast("cuda", dtype=torch.bfloat16):
        _, _, enc_out, _ = sc().compute_loss("ctc", sc().CTCLoss(blank=0, fused_head=False), model,
                                             feats, masks, tok, [64, 64], [10, 10], 0)
    assert not calls and enc_out.dtype == torch.bfloat16


def test_split_scan_planes():
    """sc_lucy_scan_fwd_split: out bitwise the plain scan's, out_dup == out, and out + out_lo is
    the fp32 h to ~2^-16 (the same gates run through the fp32 scan)."""
    ops = sc().ops
    g = torch.Generator().manual_seed(3)
    B, T, D = 2, 300, 128
    gates = (torch.randn(B, T, 7, D, generator=g) * 0.5).to(torch.bfloat16).to(DEV)
    h0 = torch.randn(B, D, generator=g).to(DEV)
    s0 = torch.randn(B, D, generator=g).to(DEV)
    _, out, s_out, _, wide = ops._scan_fwd(gates, h0, s0, False, split=True)
    _, ref, s_ref, _ = ops._scan_fwd(gates, h0, s0, False)
    assert torch.equal(out, ref) and torch.equal(s_out, s_ref)
    assert torch.equal(wide[..., D:2 * D], out)
    _, h32, _, _ = ops._scan_fwd(gates.float(), h0, s0, False)
    hs = out.float() + wide[..., 2 * D:].float()
    err = ((hs - h32).abs() / h32.abs().clamp_min(1e-3)).max().item()
    print(f"split planes: max rel |hi + lo - h32| {err:.2e}")
    assert err < 2 ** -15


@pytest.mark.parametrize("mode", ["labels", "full"])
def test_ctc_head_split_logits_match_fp32(mode, monkeypatch):
    """With the scan's [x_hi | x_hi | x_lo] buffer: "full" -- every logit from one bf16 GEMM
    against [W_hi | W_lo | W_hi] -- is the fp32 x.W + b to ~1e-5; "labels" -- the
    bf16 GEMM's fp32 logits with the emission columns (blank and each sequence's labels)
    recomputed from the split planes -- has those columns to ~1e-5 and the rest at the bf16
    operands' ~2e-3."""
    ops = sc().ops
    monkeypatch.setattr(ops, "HEAD_SPLIT", mode)
    g = torch.Generator().manual_seed(4)
    B, T, D, V = 2, 128, 256, 512
    x32 = torch.randn(B, T, D, generator=g).to(DEV)
    hi = x32.to(torch.bfloat16)
    wide = torch.cat([hi, hi, (x32 - hi.float()).to(torch.bfloat16)], -1).contiguous()
    x = wide[..., :D]
    w = (torch.randn(V, D, generator=g) * 0.05).to(DEV)
    b = (torch.randn(V, generator=g) * 0.1).to(DEV)
    tg = torch.randint(1, V, (B, 12), generator=g)
    tg[1, 9:] = 0
    imgs = (w.to(torch.bfloat16), w.t().contiguous().to(torch.bfloat16))
    _, logits = ops.ctc_head_loss(x, w, b, imgs, tg.to(DEV), [T, T], [12, 9], wide=wide)
    ref = x32.double() @ w.double().t() + b.double()
    _, l1 = ops.ctc_head_loss(x, w, b, imgs, tg.to(DEV), [T, T], [12, 9])
    e_plain = rel(l1, ref)
    for bi in range(B):
        cols = torch.unique(torch.cat([torch.zeros(1, dtype=torch.int64), tg[bi]])).to(DEV)
        e_em = rel(logits[bi][:, cols], ref[bi][:, cols])
        print(f"head ({mode}) emission-column logits rel err vs fp64: {e_em:.2e} "
              f"(bf16 operands {e_plain:.2e})")
        assert e_em < 2e-5
    e_all = rel(logits, ref)
    assert (e_all < 2e-5) if mode == "full" else (e_all <= 1.01 * e_plain)
    assert e_plain > 2e-4


def test_ctc_head_emission_side_input_matches_scattered_columns(monkeypatch):
    """"emis" (the default with the scan's split planes): bf16 logits from the bf16 GEMM and the
    emission columns to fp32 accuracy in a [B, T, U + 1] side array (sc_ctc_fwd_ex / _bwd_ex)
    against the same head with those columns scattered into fp32 logits and the plain fp32 HIP
    lattice: loss 1e-4, dW / db / dx 1e-2 in norm (bf16 logits in the row log-sum-exp and the
    softmax term of the other columns, bf16 dlogits)."""
    ops = sc().ops
    monkeypatch.setattr(ops, "HEAD_SPLIT", "emis")
    g = torch.Generator().manual_seed(7)
    B, T, D, V = 2, 160, 256, 512
    x32 = torch.randn(B, T, D, generator=g).to(DEV)
    hi = x32.to(torch.bfloat16)
    wide = torch.cat([hi, hi, (x32 - hi.float()).to(torch.bfloat16)], -1).contiguous()
    x = wide[..., :D]
    w = (torch.randn(V, D, generator=g) * 0.05).to(DEV)
    b = (torch.randn(V, generator=g) * 0.1).to(DEV)
    tg = torch.randint(1, V, (B, 14), generator=g)
    tg[1, 11:] = 0
    tg[0, 3:6] = 9   # repeats: duplicate emission columns
    tgd = tg.to(DEV)
    imgs = (w.to(torch.bfloat16), w.t().contiguous().to(torch.bfloat16))
    w1, b1 = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    loss, logits = ops.ctc_head_loss(x, w1, b1, imgs, tgd, [T, T - 20], [14, 11], wide=wide)
    assert logits.dtype == torch.bfloat16
    loss.backward()
    # reference: the bf16 logits as fp32 with the emission columns replaced by the side array's
    # values, through the plain fp32 lattice; gradients pushed through the same bf16 operands
    ex = ops._emission_logits(wide, w, b, tgd, 0, V)
    lab = ops._emission_columns(tgd, 0, V)
    # (the one-launch split rows against the cached split image: the same operand)
    lab_w = ops.split_weight_image(w)[lab]
    ex_ref = torch.bmm(wide, lab_w.transpose(1, 2), out_dtype=torch.float32) + b[lab].unsqueeze(1)
    assert torch.equal(ex, ex_ref)
    ref_logits = logits.detach().float().clone()
    ref_logits.scatter_(2, lab.unsqueeze(1).expand(B, T, lab.shape[1]), ex)
    ref_logits.requires_grad_(True)
    ref = sc().ctc_loss(ref_logits, tgd, [T, T - 20], [14, 11])
    ref.backward()
    dl = ref_logits.grad.reshape(-1, V)
    dw_ref = dl.t() @ x.float().reshape(-1, D)
    db_ref = dl.sum(0)
    print(f"emis head: loss {loss.item():.6f} vs {ref.item():.6f}; dW {rel(w1.grad, dw_ref):.2e} "
          f"db {rel(b1.grad, db_ref):.2e}")
    np.testing.assert_allclose(loss.item(), ref.item(), rtol=1e-4)
    assert rel(w1.grad, dw_ref) < 1e-2 and rel(b1.grad, db_ref) < 1e-2
