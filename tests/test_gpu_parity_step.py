"""Module- and step-level parity of the HIP path against the reference and the oracle.

* The drop-in LucyRNNtriton at the REFERENCE's own init against goldens produced by the reference
  module itself (tests/golden/module.npz: lucyrnn_triton.LucyRNNtriton under the Triton
  interpreter, fp32, 3 layers + LayerNorms + output_proj, two segments with carried state).
* One full C2-shape training step (T=1500, 6 x 512, V=1024; B reduced to 2 so the oracle finishes
  in seconds) against oracle/lucy_step.py: loss, every gradient, the post-Adam parameters.
* A 4-segment bf16-autocast carry against the fp32 oracle (the carried h stays fp32).

Tolerances (stated per element class; both sides fp32 unless noted):
  module goldens: tests.conftest.assert_ref_parity -- the GPU is at most 2x as far from the
  reference's fp64 run as the reference's own fp32 run is (measured noise: h up to 1.9e-3 after
  two segments at the reference init), and the fraction of elements within 1e-3 relative (floor
  1e-4 x max) of the reference fp32 output is pinned per tensor (MODULE_FRAC_OK: measured 1.0
  everywhere except d40_proj's first-segment logits, 0.963).  The gate normaliser x / sqrt(x^2 + 1e-6) has slope
  ~1e3 at 0, so rounding-order differences of a gate near zero are amplified.
  C2 step (well-conditioned init, see oracle_params -- the reference init is chaotic at C2
  depth even between the reference math's own fp32 and fp64 runs): loss 1e-4 relative;
  gradients ||g - g_ref|| / ||g_ref|| <= 1e-3 per tensor, north_star's tolerance (measured
  1.2e-4 ... 1.6e-4, profiles/r4_parity_measured.md).  The oracle runs CTC in fp64; the HIP
  lattice is fp32 in log space with every frame's emissions shifted by their maximum
  (csrc/ctc.hip), which holds the posteriors' error at ~1e-4 (2.5e-3 without the shift; ATen's own
  fp32 ctc_loss, the reference's criterion, is 5.2e-2 from fp64 on these logits).
  bf16 (the bench's arithmetic, split-precision output projection): gradient cosine >= 0.999 and
  norm within 1% per tensor; with a plain bf16 output projection the measured 2-5% loss of
  gradient direction is pinned per tensor (see BF16_MEASURED).
  Adam step 1: the post-step parameters equal clip + Adam restated on the GPU's own gradients
  (1e-4 relative, plus one fp32 ulp of the parameter), and wherever |g| >> Adam's eps (|g| > 1e-5,
  update ~ lr sign(g)) and >= 10x the tensor's rms gradient error they equal
  the oracle's post-step parameters (1e-8 + 2 ulp + the step's sensitivity lr eps / |g| to a
  gradient element off by its own size; no step may flip sign).
"""
import numpy as np
import pytest
import torch

from tests.conftest import assert_ref_parity, load_golden

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def sc():
    import statecatcher_amd as s
    return s


def to_np(t):
    return t.detach().double().cpu().numpy()


def assert_close_floor(got, ref, rtol=1e-3, afrac=1e-4, aabs=0.0):
    ref = np.asarray(ref, np.float64)
    np.testing.assert_allclose(to_np(got) if isinstance(got, torch.Tensor) else got, ref, rtol=rtol,
                               atol=max(aabs, afrac * max(1.0, np.abs(ref).max())))


def load_module_case(z, name):
    pre = name + "/param/"
    sd = {k[len(pre):]: torch.from_numpy(z[k]) for k in z.files if k.startswith(pre)}
    Din = sd["tracks.0.0.linear.weight"].shape[1]
    D = sd["tracks.0.0.linear.weight"].shape[0] // 7
    V = sd["output_proj.weight"].shape[0]
    L = len([k for k in sd if k.endswith(".linear.weight")])
    cfg = sc().LucyRNNConfig(input_dim=Din, hidden_dim=D, num_layers=L, vocab_size=V,
                             kernel_impl="triton", fused_ops=True, layer_norm=False)
    m = sc().LucyRNNtriton(cfg)
    m.load_state_dict(sd)   # the reference's state_dict keys, unchanged
    return m.to(DEV), L


# fraction of elements within 1e-3 relative of the reference's fp32 output, per (case, segment,
# tensor): measured on MI355X (profiles/r3_parity_measured.md) and pinned 0.005 below (the
# kernels are deterministic; the margin covers a change of GEMM accumulation order)
MODULE_FRAC_OK = {("d40_proj", 0, "logits"): 0.958}   # measured 0.9630; every other tensor 1.0000
MODULE_FRAC_DEFAULT = 0.995


@pytest.mark.parametrize("name", ["d64_init", "d64_proj", "d40_proj"])
def test_lucyrnn_triton_vs_reference_module_goldens_fp32(name):
    z = load_golden("module")
    m, L = load_module_case(z, name)
    state = None
    with torch.no_grad():
        for seg in range(2):
            x = torch.from_numpy(z[f"{name}/seg{seg}/x"]).to(DEV)
            logits, (fh, fs) = m(x, state) if state is not None else m(x)
            pre = f"{name}/seg{seg}/"
            for got, key in [(logits, "logits"), (torch.stack(fh[0]), "h"), (torch.stack(fs[0]), "s")]:
                floor = MODULE_FRAC_OK.get((name, seg, key), MODULE_FRAC_DEFAULT)
                e64, noise, frac = assert_ref_parity(to_np(got), z[pre + key], z[pre + key + "64"],
                                                     frac_ok=floor)
                print(f"{name} seg{seg} {key}: |gpu - ref64| {e64:.2e}, reference fp32 noise "
                      f"{noise:.2e}, within 1e-3 of ref fp32: {frac:.4f} (pinned >= {floor})")
            assert fh[0][0].dtype == torch.float32 and fh[0][0].is_contiguous()
            state = (fh, fs)


def test_lucyrnn_triton_vs_reference_module_goldens_bf16_autocast():
    """Same goldens under bf16 autocast (bf16 gates and layer outputs, fp32 state and carry).
    At the reference init bf16 is NOT comparable element-wise, at any layer: the k, v gates start
    near 0 (bias 0), where kv = k v / (rho^2 (rho^2 + 1e-6)) reaches ~1e5, so bf16's
    2^-9 relative rounding of k and v moves s by ~1e3 and flips sign(s), hence c = tanh(hn + s)
    and h (measured: max |dh| 1.8-1.9 in every layer).  What must hold: finite logits, |h| <= 1,
    an fp32 carried state -- and at a well-conditioned init the bf16 step tracks the fp32 oracle
    (test_c2_training_step_bf16_vs_oracle, test_four_segment_bf16_carry_vs_fp32_oracle)."""
    z = load_golden("module")
    name = "d64_proj"
    m, L = load_module_case(z, name)
    state = None
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for seg in range(2):
            x = torch.from_numpy(z[f"{name}/seg{seg}/x"]).to(DEV)
            logits, (fh, fs) = m(x, state) if state is not None else m(x)
            h = to_np(torch.stack(fh[0]))
            print(f"bf16 seg{seg}: per-layer max |dh| {np.abs(h - z[f'{name}/seg{seg}/h']).max(axis=(1, 2))}")
            assert np.isfinite(to_np(logits)).all() and np.abs(h).max() <= 1.0
            assert np.isfinite(to_np(torch.stack(fs[0]))).all()
            assert fh[0][0].dtype == torch.float32 and fs[0][0].dtype == torch.float32
            state = (fh, fs)


def test_bf16_layers_at_reference_init_match_reference_math_on_their_own_inputs(monkeypatch):
    """The bf16 path at the REFERENCE's own init, pinned numerically (verdict r5 weak item 2).
    End to end it cannot match the fp32 reference element-wise (the previous test's docstring: a
    2^-9 rounding of k or v near 0 moves s by ~1e3), so every layer is checked on its OWN inputs
    instead, both segments of the d64_proj case, state carried:
      * the gate GEMM: its bf16 gates against fp64 x W^T of the same bf16 operands, rounded to
        bf16 (one bf16 ulp, 2^-7 of the value, + 1e-6 of the largest |gate|: a value the fp32
        accumulation order puts on the other side of a rounding boundary);
      * the scan: its output h against the reference recurrence (oracle/lucy_scan.py, restating
        lucyrnn_triton.py:179-244) in fp64 on the same bf16 gates + fp32 bias and the same
        carried (h0, s0): every element within 2^-7 of the value + 2^-9 (the bf16 rounding of h
        and the fp32 state arithmetic; measured max 1.95e-3 = half a bf16 ulp at |h| ~ 1), and
        the final fp32 state s to 1e-5 of max |s| (measured <= 2.7e-7)."""
    from oracle import lucy_scan as oscan
    from statecatcher_amd import ops as o
    z = load_golden("module")
    name = "d64_proj"
    m, L = load_module_case(z, name)
    seen = {"gemm": [], "scan": []}
    orig_proj, orig_scan = o.proj_fwd, o._scan_fwd

    def proj(x, w):
        out = orig_proj(x, w)
        seen["gemm"].append((x.detach().clone(), w.detach().clone(), out.detach().clone()))
        return out

    def scan(gates, h0, s0, need, bias=None, **kw):
        res = orig_scan(gates, h0, s0, need, bias, **kw)
        seen["scan"].append((gates.detach().clone(), h0.detach().float().clone(),
                             s0.detach().float().clone(), None if bias is None else bias.clone(),
                             res[1].detach().clone(), res[2].detach().clone()))
        return res
    monkeypatch.setattr(o, "proj_fwd", proj)
    monkeypatch.setattr(o, "_scan_fwd", scan)
    state = None
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for seg in range(2):
            x = torch.from_numpy(z[f"{name}/seg{seg}/x"]).to(DEV)
            _, state = m(x, state) if state is not None else m(x)
    torch.cuda.synchronize()
    assert len(seen["scan"]) == 2 * L and len(seen["gemm"]) >= 2 * L
    for x, w, out in seen["gemm"]:
        ref = (x.double() @ w.double().t()).to(torch.bfloat16).double()
        err = (out.double() - ref).abs()
        assert bool((err <= ref.abs() * 2.0 ** -7 + 1e-6 * float(ref.abs().max())).all()), \
            float(err.max())
    for i, (g, h0, s0, bias, out, s_out) in enumerate(seen["scan"]):
        B, T, D, _ = o.gate_layout(g)
        g32 = g.float()
        if g32.dim() == 5:   # step-blocked [B,T,D/64,7,64] -> the reference's [B,T,7,D]
            g32 = g32.permute(0, 1, 3, 2, 4).reshape(B, T, 7, D)
        if bias is not None:
            g32 = g32 + bias.view(1, 1, 7, D)
        ref_out, ref_s = oscan.lucy_scan_fwd(to_np(g32), to_np(h0), to_np(s0))
        got = to_np(out)
        e = np.abs(got - ref_out)
        ok = e <= np.abs(ref_out) * 2.0 ** -7 + 2.0 ** -9
        es = np.abs(to_np(s_out) - ref_s)
        srel = float(es.max() / max(np.abs(ref_s).max(), 1e-30))
        print(f"layer call {i}: h within tol {ok.mean():.5f} (max err {e.max():.2e}), s max rel "
              f"{srel:.2e}")
        assert ok.all() and srel <= 1e-5


# ----------------------------------------------------------------------- C2 training step ---
L6, D512, V1024, DIN = 6, 512, 1024, 80


def oracle_params():
    """The reference init (xavier + gate biases, oracle.lucy_step.init_params) made
    well-conditioned: gate planes z..alpha get 0.1x weights and biases of +-3 (as
    test_gpu_model.condition_).  At the reference init itself the C2-depth forward is CHAOTIC:
    the oracle's own fp32 and fp64 runs (B=2, T=1500, 6 x 512) differ by a mean |dh| of 0.69 in
    layer 5 and by up to 2.26 in the logits (scale 1.7) -- bf16 or fp32, no implementation can
    match it element-wise there.  Conditioned, fp32 vs fp64 agree to 1e-6."""
    from oracle import lucy_step
    p = lucy_step.init_params(L6, DIN, D512, V1024, seed=11)
    rng = np.random.default_rng(3)
    for l in range(L6):
        W = p[f"W{l}"].reshape(7, D512, -1)
        b = p[f"b{l}"].reshape(7, D512)
        W[1:] *= 0.1
        b[1:] = 3.0 * (rng.integers(0, 2, (6, D512)) * 2 - 1)
    return p


def model_from(p):
    cfg = sc().build_lucyrnn_config(DIN, D512, L6, V1024)
    model = sc().ASRModel(None, cfg, vocab_size=V1024, feat_dim=DIN, proj_dim=-1)
    enc = model.encoder
    with torch.no_grad():
        for l in range(L6):
            enc.tracks[0][l].linear.weight.copy_(torch.from_numpy(p[f"W{l}"]))
            enc.tracks[0][l].linear.bias.copy_(torch.from_numpy(p[f"b{l}"]))
            if l < L6 - 1:
                enc.norms[0][l].weight.copy_(torch.from_numpy(p[f"g{l}"]))
                enc.norms[0][l].bias.copy_(torch.from_numpy(p[f"be{l}"]))
        enc.output_proj.weight.copy_(torch.from_numpy(p["Wo"]))
        enc.output_proj.bias.copy_(torch.from_numpy(p["bo"]))
    return model.to(DEV)


def oracle_key(name):
    parts = name.split(".")
    if parts[1] == "output_proj":
        return "Wo" if parts[2] == "weight" else "bo"
    l = int(parts[3])
    if parts[1] == "tracks":
        return f"W{l}" if parts[5] == "weight" else f"b{l}"
    return f"g{l}" if parts[4] == "weight" else f"be{l}"


def step_inputs(B, T, seed):
    rng = np.random.default_rng(seed)
    feats = rng.standard_normal((B, T, DIN)).astype(np.float32)
    U = rng.integers(50, 151, B)
    tok = rng.integers(1, V1024, (B, int(U.max())))
    for b in range(B):
        tok[b, U[b]:] = 0
    return feats, tok, U


def test_c2_training_step_fp32_vs_oracle():
    from oracle import lucy_step
    from statecatcher_amd.train import SegmentTrainer
    B, T = 2, 1500
    p = oracle_params()
    model = model_from(p)
    feats, tok, U = step_inputs(B, T, 5)
    in_lens = np.full(B, T)
    opt = torch.optim.Adam(model.parameters(), lr=3e-4, fused=True)
    tr = SegmentTrainer(model, sc().CTCLoss(blank=0, zero_infinity=True), opt, max_grad_norm=50.0)
    loss, _, enc_out, _ = sc().compute_loss("ctc", tr.criterion, model, torch.from_numpy(feats).to(DEV),
                                            torch.ones(B, T, dtype=torch.bool, device=DEV),
                                            torch.from_numpy(tok).to(DEV), in_lens.tolist(),
                                            U.tolist(), 0)
    enc_out.retain_grad()
    loss.backward()
    grads = {oracle_key(k): v.grad.detach().double().cpu().numpy() for k, v in model.named_parameters()}
    # the CTC gradient on these very logits against ATen fp64, next to ATen fp32 (the reference's
    # criterion) on the same logits: the HIP lattice must be at least as accurate
    lg = enc_out.detach().cpu()
    errs = {}
    for dt in (torch.float64, torch.float32):
        xr = lg.to(dt).requires_grad_(True)
        torch.nn.CTCLoss(blank=0, zero_infinity=True)(xr.log_softmax(-1).transpose(0, 1),
                                                      torch.from_numpy(tok), in_lens.tolist(),
                                                      U.tolist()).backward()
        errs[dt] = xr.grad.double().numpy()
    r64 = errs[torch.float64]
    hip = enc_out.grad.double().cpu().numpy()
    e_hip = np.linalg.norm(hip - r64) / np.linalg.norm(r64)
    e_aten = np.linalg.norm(errs[torch.float32] - r64) / np.linalg.norm(r64)
    print(f"dlogits rel err vs ATen fp64: HIP {e_hip:.2e}, ATen fp32 {e_aten:.2e}")
    assert e_hip <= max(e_aten, 1e-4)
    tr._clip_and_step()
    p0 = {k: v.copy() for k, v in p.items()}
    ref_loss, _, ref_grads, _ = lucy_step.train_step(p, feats, tok, in_lens, U, L6, D512)
    print(f"fp32 loss {loss.item():.6f} oracle {ref_loss:.6f}")
    np.testing.assert_allclose(loss.item(), ref_loss, rtol=1e-4)
    assert set(grads) == set(ref_grads)
    rels = {}
    for k, g in grads.items():
        rg = np.asarray(ref_grads[k], np.float64)
        rels[k] = np.linalg.norm(g - rg) / np.linalg.norm(rg)
        print(f"fp32 grad {k}: rel {rels[k]:.2e} norm {np.linalg.norm(rg):.3e} "
              f"max-err/max {np.abs(g - rg).max() / np.abs(rg).max():.2e}")
    assert max(rels.values()) < 1e-3, rels
    # the encoder's backward on its own, free of CTC-lattice noise: the oracle fed the GPU's own
    # d loss / d logits must give every encoder gradient to 1e-3 (north_star tolerance)
    _, _, x_o, (caches_o, h_o, s_o) = lucy_step.forward(p0, feats, L6, D512)   # pre-Adam weights
    enc_g = lucy_step.encoder_backward(p0, hip.astype(np.float32), x_o, caches_o, h_o, s_o, L6, D512)
    e_enc = {k: np.linalg.norm(grads[k] - enc_g[k]) / np.linalg.norm(enc_g[k]) for k in enc_g}
    print("fp32 encoder backward on the GPU's dlogits, rel: " +
          " ".join(f"{k} {v:.1e}" for k, v in e_enc.items()))
    assert max(e_enc.values()) < 1e-3, e_enc
    # clip + Adam step 1, restated on OUR gradients, equals the fused step exactly; and where the
    # gradient is far above Adam's eps (update ~ lr sign(g)) it equals the oracle's update
    tot = np.sqrt(sum(float((g ** 2).sum()) for g in grads.values()))
    coef = min(1.0, 50.0 / (tot + 1e-6))
    for k, v in model.named_parameters():
        ok = oracle_key(k)
        upd = to_np(v) - p0[ok]
        g = grads[ok] * coef
        mine = -3e-4 * (0.1 * g / 0.1) / (np.sqrt(0.001 * g * g / 0.001) + 1e-8)
        ulp = np.spacing(np.abs(p0[ok]).astype(np.float32)).astype(np.float64)   # fp32 params
        assert (np.abs(upd - mine) <= 1e-4 * np.abs(mine) + ulp).all(), k
        ref_upd = p[ok].astype(np.float64) - p0[ok]
        # elements whose gradient stands clear of the tensor's rms gradient error (so its sign is
        # determined) and of Adam's eps
        rg = np.asarray(ref_grads[ok], np.float64)
        err_rms = np.linalg.norm(grads[ok] - rg) / np.sqrt(rg.size)
        big = (np.abs(rg) > 10 * err_rms) & (np.abs(rg) * coef > 1e-5)
        # d/dg of lr g / (|g| + eps) is lr eps / |g|^2: a gradient element off by up to its own
        # size moves the step by <= lr eps / |g| (3e-7 at |g| = 1e-5); a sign flip would be 6e-4
        sens = 3e-4 * 1e-8 / (np.abs(ref_grads[ok]) * coef)[big]
        same = np.abs(upd - ref_upd)[big] <= 1e-8 + 2 * ulp[big] + sens
        assert same.all(), (k, int((~same).sum()))


# bf16 step vs the fp32 oracle with the output projection in plain bf16 (CTCLoss(fused_head=False):
# bf16 operands, bf16 logits), measured on MI355X (profiles/r3_parity_measured.md): per tensor
# (gradient cosine, norm ratio).  The 2-5% loss is the output projection's rounding alone -- of its
# operands or of the logits -- which shifts CTC's alignment posteriors coherently over T = 1500
# frames (tools/bf16_logits_diag.py reproduces these values on the CPU oracle; unbiased noise of
# the same size costs nothing).  The kernels are deterministic, so these repeat exactly; the
# bounds leave 0.006 of cosine and 0.02 of norm ratio for a change of GEMM accumulation order.
BF16_MEASURED = {
    "encoder.tracks.0.0.linear.weight": (0.9999, 1.0005),
    "encoder.tracks.0.0.linear.bias": (0.9886, 0.9710),
    "encoder.tracks.0.1.linear.weight": (0.9808, 0.9508),
    "encoder.tracks.0.1.linear.bias": (0.9809, 0.9503),
    "encoder.tracks.0.2.linear.weight": (0.9754, 0.9456),
    "encoder.tracks.0.2.linear.bias": (0.9754, 0.9461),
    "encoder.tracks.0.3.linear.weight": (0.9732, 0.9687),
    "encoder.tracks.0.3.linear.bias": (0.9732, 0.9688),
    "encoder.tracks.0.4.linear.weight": (0.9771, 0.9620),
    "encoder.tracks.0.4.linear.bias": (0.9771, 0.9619),
    "encoder.tracks.0.5.linear.weight": (0.9761, 0.9803),
    "encoder.tracks.0.5.linear.bias": (0.9762, 0.9808),
    "encoder.norms.0.0.weight": (0.9968, 0.9895),
    "encoder.norms.0.0.bias": (0.9971, 0.9863),
    "encoder.norms.0.1.weight": (0.9856, 0.9573),
    "encoder.norms.0.1.bias": (0.9855, 0.9604),
    "encoder.norms.0.2.weight": (0.9730, 0.9857),
    "encoder.norms.0.2.bias": (0.9724, 0.9825),
    "encoder.norms.0.3.weight": (0.9761, 0.9532),
    "encoder.norms.0.3.bias": (0.9762, 0.9569),
    "encoder.norms.0.4.weight": (0.9768, 0.9778),
    "encoder.norms.0.4.bias": (0.9773, 0.9764),
    "encoder.output_proj.weight": (0.9755, 0.9746),
    "encoder.output_proj.bias": (0.9754, 0.9747),
}
BF16_COS_MARGIN, BF16_RATIO_MARGIN = 0.006, 0.02


@pytest.mark.parametrize("fused_head", [True, False])
def test_c2_training_step_bf16_vs_oracle(fused_head):
    """The bench's arithmetic (bf16 autocast GEMMs, bf16 gates, fp32 state): loss within 1e-2
    relative of the fp32 oracle.  fused_head (the default, what the bench runs): the last scan
    writes [x_hi | x_hi | x_lo] and the output projection is one bf16 GEMM against
    [W_hi | W_lo | W_hi] with fp32 logits (ops.CTCHeadFn) -- every gradient's cosine >= 0.999 and
    norm within 1% of the fp32 oracle (measured 1.0000 and <= 0.3%, profiles/r4_parity_measured.md).
    Without it, per tensor within the margins of BF16_MEASURED."""
    from oracle import lucy_step
    B, T = 2, 1500
    p = oracle_params()
    model = model_from(p)
    feats, tok, U = step_inputs(B, T, 6)
    in_lens = np.full(B, T)
    crit = sc().CTCLoss(blank=0, zero_infinity=True, fused_head=fused_head)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss, _, _, _ = sc().compute_loss("ctc", crit, model,
                                          torch.from_numpy(feats).to(DEV),
                                          torch.ones(B, T, dtype=torch.bool, device=DEV),
                                          torch.from_numpy(tok).to(DEV), in_lens.tolist(), U.tolist(), 0)
    loss.backward()
    ref_loss, _, ref_grads, _ = lucy_step.train_step(p, feats, tok, in_lens, U, L6, D512)
    print(f"bf16 (fused_head={fused_head}) loss {loss.item():.6f} oracle {ref_loss:.6f}")
    np.testing.assert_allclose(loss.item(), ref_loss, rtol=1e-2)
    bad = []
    for k, v in model.named_parameters():
        g = to_np(v.grad).ravel()
        rg = np.asarray(ref_grads[oracle_key(k)], np.float64).ravel()
        cos = float(g @ rg / (np.linalg.norm(g) * np.linalg.norm(rg)))
        ratio = float(np.linalg.norm(g) / np.linalg.norm(rg))
        print(f"bf16 (fused_head={fused_head}) grad {k}: cos {cos:.4f} norm ratio {ratio:.4f}")
        if fused_head:
            ok = cos >= 0.999 and abs(ratio - 1.0) <= 0.01
        else:
            mc, mr = BF16_MEASURED[k]
            ok = cos >= mc - BF16_COS_MARGIN and abs(ratio - mr) <= BF16_RATIO_MARGIN
        if not ok:
            bad.append((k, cos, ratio))
    assert not bad, bad


def test_four_segment_bf16_carry_vs_fp32_oracle():
    """4 consecutive segments under bf16 autocast, state carried (detached) between them, against
    the fp32 oracle carrying the same state: the carried h is the scan's fp32 h_last, so the
    drift after 4 segments is bf16 GEMM/gate rounding only (no bf16 state rounding)."""
    from oracle import lucy_step
    B, T = 2, 1500
    p = oracle_params()
    model = model_from(p)
    state_ref, state = None, None
    for seg in range(4):
        feats, _, _ = step_inputs(B, T, 100 + seg)
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
            logits, state = model(torch.from_numpy(feats).to(DEV),
                                  torch.ones(B, T, dtype=torch.bool, device=DEV), state)
        ref_logits, state_ref, _, _ = lucy_step.forward(p, feats, L6, D512, state_ref)
        # the first frames of a segment depend on the carried state
        el = np.abs(to_np(logits)[:, :32] - ref_logits[:, :32]) / np.abs(ref_logits).max()
        print(f"seg {seg}: first-32-frame logits err max {el.max():.3e} mean {el.mean():.3e}")
        assert el.max() < 2e-2
        h = np.stack([to_np(t) for t in state[0][0]])
        s = np.stack([to_np(t) for t in state[1][0]])
        assert state[0][0][0].dtype == torch.float32
        eh = np.abs(h - np.stack(state_ref[0]))
        es = np.abs(s - np.stack(state_ref[1])) / np.maximum(1.0, np.abs(np.stack(state_ref[1])))
        print(f"seg {seg}: h err max {eh.max():.3e} mean {eh.mean():.3e}; s rel err max {es.max():.3e}")
        assert eh.mean() < 5e-3 and np.percentile(eh, 99) < 5e-2
        assert es.mean() < 5e-3
