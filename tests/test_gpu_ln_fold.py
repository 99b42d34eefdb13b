"""GPU parity of the inter-layer LayerNorm folded into the next gate projection (csrc/ln_fold.hip,
ops.LucyCellLNFn), which replaces nn.LayerNorm + LinearSafe (lucyrnn_triton.py:96-97, :136-137,
:20-25) under bf16 autocast, in both of its forms (the tests switch them on):
  mode 1 (SC_LN_FOLD=1, round 5): the scans apply it (sc_lucy_scan_fwd_ln / _bwd_ln rebuild the
         gates from block records);
  mode 2 (SC_LN_FOLD=2, round 6): the gate GEMM applies it (sc_gemm_tn_ln_bf16: row statistics
         from the streaming rows, normalised gates out), the backward scan only scales.

* sc_gemm_tn_ln_bf16 against fp64 torch (LN(h) W^T - W beta from the same bf16 h) and its
  statistics against torch's.

* The folded images (W'' = bf16(gamma W - shift)), b' and r against torch on the same fp32
  values.
* One LayerNorm + LucyRNN layer, fold against the unfused bf16 path (LayerNorm kernel -> bf16 ->
  gate GEMM -> scan) and both against the fp32 path of the same module: the fold is at least as
  close to fp32 as the unfused bf16 path (1.5x + floor), outputs, states and every gradient
  (d input, dW, db, dgamma, dbeta, dh0, ds0).
* A 6 x 512 stack (config C2's model) under autocast: loss and every parameter gradient of the
  fold against fp32, no further than the unfused bf16 stack (2x + floor).
Both use conditioned gates (condition_): at xavier init the reference's gate normalisation makes
any two precisions of the model differ at O(1) (tests/test_gpu_model.py's docstring)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def ops():
    from statecatcher_amd import ops as o
    return o


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return float((a @ b) / max(float(a.norm() * b.norm()), 1e-30))


def test_fold_images_match_torch():
    g = torch.Generator().manual_seed(1)
    D = 512
    w = (torch.randn(7 * D, D, generator=g) * 0.03).to(DEV)
    b = (torch.randn(7 * D, generator=g) * 0.1).to(DEV)
    gam = (1.0 + 0.2 * torch.randn(D, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(D, generator=g)).to(DEV)
    (img, img_t, bprime, rowsum, r_img), = ops().fold_images([(w, b, gam, bet, D, D, True)])
    torch.cuda.synchronize()
    gw = gam * w                                   # exact fp32 products, as the kernels form them
    shift = gw.double().mean(1)
    ref = (gw - shift.float().unsqueeze(1)).to(torch.bfloat16)
    got = ops().step_blocked_rows(img, D, inverse=True)
    # one shift's last-bit difference (summation order) may move a rounding boundary
    assert (got.float() - ref.float()).abs().max() <= 2.0 ** -7 * ref.float().abs().max()
    assert (got != ref).float().mean() < 1e-4
    assert torch.equal(img_t, img.t())
    torch.testing.assert_close(bprime.double(), (b.double() + w.double() @ bet.double()),
                               rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rowsum.double(), got.double().sum(1), rtol=0, atol=1e-6)
    assert float(rowsum.abs().max()) < 1e-2 * float(gw.abs().sum(1).max())
    # r in the image's (step-blocked) row order: the row sums of the image's own rows
    torch.testing.assert_close(r_img.double(), img.double().sum(1), rtol=0, atol=1e-6)


def _set_mode(monkeypatch, mode):
    from statecatcher_amd import lucyrnn_triton as lt
    o = ops()
    monkeypatch.setattr(o, "USE_LN_FOLD", mode != 0)
    monkeypatch.setattr(o, "LN_FOLD_MODE", mode)
    monkeypatch.setattr(lt, "LN_FOLD_MODE", mode)


@pytest.mark.parametrize("M", [48000, 1000, 7])
def test_gemm_tn_ln_vs_torch(M):
    """sc_gemm_tn_ln_bf16 = rstd (h W''^T - mean r) against fp64 torch's LN(h) W^T - W beta on the
    same bf16 h (the scan adds b' = b + W beta), at C2's shape, a ragged panel and fewer rows than
    a fragment; the (rstd, mean) it writes against torch's biased statistics.  Tolerance: the
    bf16 output rounding (2^-8 of each value) plus the W'' image's bf16 rounding, which the
    unfused path pays on LN(h) instead (1e-2 of the largest |C|)."""
    g = torch.Generator().manual_seed(M)
    D = 512
    w = (torch.randn(7 * D, D, generator=g) * 0.03).to(DEV)
    b = (torch.randn(7 * D, generator=g) * 0.1).to(DEV)
    gam = (1.0 + 0.2 * torch.randn(D, generator=g)).to(DEV)
    bet = (0.1 * torch.randn(D, generator=g)).to(DEV)
    h = (torch.randn(M, D, generator=g) * 0.4 + 0.3 * torch.randn(M, 1, generator=g)).to(DEV) \
        .to(torch.bfloat16)
    (img, _, bprime, _, r_img), = ops().fold_images([(w, b, gam, bet, D, D, False)])
    c, stat = ops().gemm_tn_ln(h, img, r_img, 1e-5)
    torch.cuda.synchronize()
    h64 = h.double()
    mean = h64.mean(1, keepdim=True)
    var = h64.var(1, unbiased=False, keepdim=True)
    y = (h64 - mean) / torch.sqrt(var + 1e-5) * gam.double() + bet.double()
    wsb = ops().step_blocked_rows(w, D).double()           # the image's row order
    ref = y @ wsb.t() - (wsb @ bet.double())
    err = (c.double() - ref).abs()
    tol = ref.abs() * 2.0 ** -8 + 1e-2 * float(ref.abs().max())
    print(f"M={M}: max err {float(err.max()):.3e} (|C| max {float(ref.abs().max()):.2f}), rel "
          f"Frobenius {rel(c, ref):.2e}")
    assert bool((err <= tol).all())
    assert rel(c, ref) <= 5e-3
    torch.testing.assert_close(stat[:, 1].double(), mean[:, 0], rtol=0, atol=2e-6)
    torch.testing.assert_close(stat[:, 0].double(), 1.0 / torch.sqrt(var[:, 0] + 1e-5),
                               rtol=2e-5, atol=0)


def condition_(m, D, gen):
    """Well-conditioned gates (tests/test_gpu_model.py's module docstring): the reference's
    x / sqrt(x^2 + 1e-6) gate normalisation flips any gate within ~1e-5 of zero between two
    precisions, so at xavier init bf16 and fp32 runs of one model differ by O(1) after a few
    layers.  |bias| = 3 on z, k, v, h_pre, decay, alpha keeps them away from zero."""
    with torch.no_grad():
        for cell in m.tracks[0]:
            W, b = cell.linear.weight.view(7, D, -1), cell.linear.bias.view(7, D)
            for gi in (1, 2, 3, 4, 5, 6):
                W[gi] *= 0.1
                b[gi] = 3.0 * (torch.randint(0, 2, (D,), generator=gen).float() * 2 - 1).to(b.device)


def _layer_pair(D=512, B=2, T=200, seed=3):
    """(module with 2 layers, input x [B,T,80]) at a trained-like spread of LN parameters."""
    from statecatcher_amd import LucyRNNConfig, LucyRNNtriton
    torch.manual_seed(seed)
    cfg = LucyRNNConfig(input_dim=80, hidden_dim=D, num_layers=2, vocab_size=128, fused_ops=True,
                        layer_norm=False)
    m = LucyRNNtriton(cfg).to(DEV)
    condition_(m, D, torch.Generator().manual_seed(seed + 100))
    with torch.no_grad():
        m.norms[0][0].weight.normal_(1.0, 0.2)
        m.norms[0][0].bias.normal_(0.0, 0.1)
        m.output_proj.weight.normal_(0, 0.05)
    x = torch.randn(B, T, 80, device=DEV)
    return m, x


def _run(m, x, autocast):
    m.zero_grad(set_to_none=True)
    xd = x.clone().requires_grad_(True)
    B, D = x.shape[0], m.config.hidden_dim
    h0 = [[(0.5 * torch.randn(B, D, device=DEV, generator=torch.Generator(DEV).manual_seed(5 + l)))
           .requires_grad_(True) for l in range(2)]]
    s0 = [[(0.5 * torch.randn(B, D, device=DEV, generator=torch.Generator(DEV).manual_seed(9 + l)))
           .requires_grad_(True) for l in range(2)]]
    R = torch.randn(x.shape[0], x.shape[1], m.config.vocab_size, device=DEV,
                    generator=torch.Generator(DEV).manual_seed(7))
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        logits, (fh, fs) = m(xd, ([h0[0][:]], [s0[0][:]]))
        loss = (logits.float() * R).sum() + fh[0][1].sum() + fs[0][1].square().sum()
    loss.backward()
    out = {"logits": logits.detach().float(), "h_last": fh[0][1].detach().float(),
           "s_last": fs[0][1].detach().float(), "dx": xd.grad.float(),
           "dh0_1": h0[0][1].grad.float(), "ds0_1": s0[0][1].grad.float()}
    for n, p in m.named_parameters():
        out["d " + n] = p.grad.detach().float().clone()
    return out


@pytest.mark.parametrize("mode", [1, 2])
def test_fold_layer_vs_unfused_and_fp32(monkeypatch, mode):
    _set_mode(monkeypatch, mode)   # (opt-in: SC_LN_FOLD=1 / 2)
    m, x = _layer_pair()
    ref32 = _run(m, x, autocast=False)
    folded = _run(m, x, autocast=True)
    _set_mode(monkeypatch, 0)
    plain = _run(m, x, autocast=True)
    lines, bad = [], []
    for k in ref32:
        ef, ep = rel(folded[k], ref32[k]), rel(plain[k], ref32[k])
        lines.append(f"{k}: fold {ef:.2e} unfused {ep:.2e}")
        if ef > max(1.5 * ep, 5e-3):   # (both carry bf16 noise of their own rounding points)
            bad.append((k, ef, ep))
    print("LN fold vs fp32 (rel. Frobenius): " + "; ".join(lines))
    assert not bad, bad


@pytest.mark.parametrize("mode", [1, 2])
def test_fold_engaged_and_no_layernorm_launch(monkeypatch, mode):
    """The bf16 forward of a 3-layer stack takes LucyCellLNFn for layers 1 and 2 and never
    launches the LayerNorm kernel."""
    from statecatcher_amd import LucyRNNConfig, LucyRNNtriton
    calls = {"ln": 0, "fold": 0}
    o = ops()
    _set_mode(monkeypatch, mode)
    orig_ln, orig_fold = o.LayerNormFn.apply, o.LucyCellLNFn.apply

    def ln(*a):
        calls["ln"] += 1
        return orig_ln(*a)

    def fold(*a):
        calls["fold"] += 1
        return orig_fold(*a)
    monkeypatch.setattr(o.LayerNormFn, "apply", ln)
    monkeypatch.setattr(o.LucyCellLNFn, "apply", fold)
    torch.manual_seed(0)
    m = LucyRNNtriton(LucyRNNConfig(input_dim=80, hidden_dim=512, num_layers=3, vocab_size=64,
                                    fused_ops=True, layer_norm=False)).to(DEV)
    x = torch.randn(1, 64, 80, device=DEV)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        m(x)
    assert calls == {"ln": 0, "fold": 2}


@pytest.mark.parametrize("mode", [1, 2])
def test_c2_stack_fold_vs_unfused(monkeypatch, mode):
    """6 x 512, V = 1024, T = 1500, B = 2 with the CTC criterion, conditioned gates: the loss and
    every parameter gradient of the folded bf16 stack against the fp32 run of the same model, no
    further from it than the unfused bf16 stack is (2x + floor)."""
    from statecatcher_amd.model import ASRModel, CTCLoss, build_lucyrnn_config, compute_loss
    torch.manual_seed(11)
    V, B, T = 1024, 2, 1500
    model = ASRModel(None, build_lucyrnn_config(80, 512, 6, V), vocab_size=V, feat_dim=80,
                     proj_dim=-1).to(DEV)
    condition_(model.encoder, 512, torch.Generator().manual_seed(12))
    with torch.no_grad():
        model.encoder.output_proj.weight.normal_(0, 0.02)
        for ln in model.encoder.norms[0]:
            ln.weight.normal_(1.0, 0.1)
            ln.bias.normal_(0.0, 0.05)
    g = torch.Generator().manual_seed(7)
    feats = torch.randn(B, T, 80, generator=g).to(DEV)
    tok = torch.randint(1, V, (B, 150), generator=g).to(DEV)
    crit = CTCLoss(blank=0, zero_infinity=True)

    def run(amp):
        model.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss, _, _, _ = compute_loss("ctc", crit, model, feats,
                                         torch.ones(B, T, dtype=torch.bool, device=DEV), tok,
                                         [T, T], [150, 97], 0)
        loss.backward()
        return float(loss), {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    _set_mode(monkeypatch, mode)
    l32, g32 = run(False)
    lf, gf = run(True)
    _set_mode(monkeypatch, 0)
    lp, gp = run(True)
    print(f"C2 stack loss fp32 {l32:.6f} fold {lf:.6f} unfused {lp:.6f}")
    assert abs(lf - l32) <= max(2 * abs(lp - l32), 1e-3 * abs(l32))
    errs, bad = [], []
    for n in g32:
        ef, ep = rel(gf[n], g32[n]), rel(gp[n], g32[n])
        errs.append((ef, ep, n))
        if ef > max(2.0 * ep, 2e-2):
            bad.append((n, ef, ep))
    errs.sort(reverse=True)
    print("largest gradient errors vs fp32 (fold / unfused): "
          + "; ".join(f"{n} {ef:.2e} / {ep:.2e}" for ef, ep, n in errs[:6]))
    assert not bad, bad
