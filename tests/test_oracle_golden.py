"""Pin the CPU oracle against fixtures produced by the reference itself (CPU, no GPU)."""
import numpy as np
import pytest
import torch

from oracle import ctc as octc
from oracle import decode as odec
from oracle import lucy_scan as oscan
from tests.conftest import cases, load_golden


@pytest.mark.parametrize("name", cases(load_golden("scan_fwd"), "gates"))
def test_scan_fwd_vs_reference_triton(name):
    z = load_golden("scan_fwd")
    out, s = oscan.lucy_scan_fwd(z[name + "/gates"], z[name + "/h0"], z[name + "/s0"])
    ref_out = z[name + "/out"]
    ref_s = z[name + "/s_out"]
    # reference kernel is fp32: 1e-3 relative (north_star tolerance) with a small abs floor
    np.testing.assert_allclose(out, ref_out, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(s, ref_s, rtol=1e-3, atol=1e-4 * max(1.0, np.abs(ref_s).max()) * 1e-2)


def test_scan_fwd_fp32_oracle_matches_reference_tightly():
    z = load_golden("scan_fwd")
    out, s = oscan.lucy_scan_fwd(z["realistic/gates"], z["realistic/h0"], z["realistic/s0"],
                                 dtype=np.float32)
    np.testing.assert_allclose(out, z["realistic/out"], rtol=2e-5, atol=2e-6)


def test_scan_carry_contiguous_and_aliasing_bug_documented():
    z = load_golden("scan_fwd")
    out1, s1 = oscan.lucy_scan_fwd(z["carry/g1"], np.zeros((3, 16)), np.zeros((3, 16)))
    np.testing.assert_allclose(out1, z["carry/out1"], rtol=1e-4, atol=1e-6)
    out2, s2 = oscan.lucy_scan_fwd(z["carry/g2"], out1[:, -1], s1)
    np.testing.assert_allclose(out2, z["carry/out2_contig"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(s2, z["carry/s2_contig"], rtol=1e-4, atol=1e-5)
    # the reference's strided h0 view corrupts rows b >= 1 but not b = 0
    alias = z["carry/out2_aliased"]
    np.testing.assert_allclose(alias[0], z["carry/out2_contig"][0], rtol=1e-6)
    assert np.abs(alias[1:] - z["carry/out2_contig"][1:]).max() > 1e-3


@pytest.mark.parametrize("name", cases(load_golden("scan_bwd"), "dgates"))
def test_scan_bwd_vs_autograd(name):
    zf = load_golden("scan_fwd")
    zb = load_golden("scan_bwd")
    g, h0, s0 = zf[name + "/gates"], zf[name + "/h0"], zf[name + "/s0"]
    dg, dh0, ds0 = oscan.lucy_scan_bwd(g, h0, s0, zb[name + "/dout"], zb[name + "/ds_last"])
    ref = zb[name + "/dgates"]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(dg, ref, rtol=1e-7, atol=1e-9 * scale)
    np.testing.assert_allclose(dh0, zb[name + "/dh0"], rtol=1e-7, atol=1e-12)
    np.testing.assert_allclose(ds0, zb[name + "/ds0"], rtol=1e-7, atol=1e-12)


def test_scan_bwd_autograd_forward_matches_reference():
    """The fp64 restatement that produced the bwd fixtures agrees with the reference forward."""
    zf = load_golden("scan_fwd")
    zb = load_golden("scan_bwd")
    for name in cases(zb, "dgates"):
        np.testing.assert_allclose(zb[name + "/out64"], zf[name + "/out"], rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("name", ["small", "t1"])
def test_decay_scan_vs_reference_triton(name):
    z = load_golden("decay_scan")
    s = oscan.decay_scan(z[name + "/kv"], z[name + "/decay"])
    np.testing.assert_allclose(s, z[name + "/s_all"], rtol=1e-6, atol=1e-6)


def test_decay_scan_bwd_vs_autograd():
    rng = np.random.default_rng(0)
    kv = rng.standard_normal((2, 17, 5))
    dec = 1 / (1 + np.exp(-rng.standard_normal((2, 17, 5))))
    dout = rng.standard_normal((2, 17, 5))
    tk = torch.tensor(kv, requires_grad=True)
    td = torch.tensor(dec, requires_grad=True)
    s = torch.zeros(2, 5, dtype=torch.float64)
    outs = []
    for t in range(17):
        s = td[:, t] * s + tk[:, t]
        outs.append(s)
    (torch.stack(outs, 1) * torch.tensor(dout)).sum().backward()
    s_all = oscan.decay_scan(kv, dec, dtype=np.float64)
    dkv, ddec = oscan.decay_scan_bwd(dec, s_all, dout)
    np.testing.assert_allclose(dkv, tk.grad.numpy(), rtol=1e-10)
    np.testing.assert_allclose(ddec, td.grad.numpy(), rtol=1e-10, atol=1e-14)


@pytest.mark.parametrize("name", cases(load_golden("ctc"), "logits"))
def test_ctc_vs_aten(name):
    z = load_golden("ctc")
    nll, grad = octc.ctc_loss_grad(z[name + "/logits"], z[name + "/targets"], z[name + "/in_lens"],
                                   z[name + "/tgt_lens"], blank=0, logits=True)
    ref = z[name + "/nll"]
    fin = np.isfinite(ref)
    assert np.array_equal(fin, np.isfinite(nll))
    np.testing.assert_allclose(nll[fin], ref[fin], rtol=1e-10)
    # per-sample grads (zero_infinity=True zeroes infeasible samples)
    g = np.where(np.isfinite(nll)[:, None, None], grad, 0.0)
    np.testing.assert_allclose(g, z[name + "/sum_grad"], rtol=1e-8, atol=1e-12)
    # mean reduction with zero_infinity
    loss = octc.ctc_mean_zero_inf(nll, z[name + "/tgt_lens"])
    np.testing.assert_allclose(loss, float(z[name + "/mean_loss"]), rtol=1e-10)
    sc = octc.ctc_mean_grad_scale(nll, z[name + "/tgt_lens"])
    gm = np.where(np.isfinite(nll)[:, None, None], grad, 0.0) * sc[:, None, None]
    np.testing.assert_allclose(gm, z[name + "/mean_grad"], rtol=1e-8, atol=1e-13)


def _split(counts, flat):
    out, o = [], 0
    for c in counts:
        out.append(list(flat[o:o + c]))
        o += c
    return out


@pytest.mark.parametrize("pref", ["ties", "big"])
def test_greedy_vs_reference_decoder(pref):
    z = load_golden("greedy")
    dec = odec.ctc_greedy(z[pref + "_lp"], z[pref + "_in_lens"], blank=0)
    assert dec == _split(z[pref + "_counts"], z[pref + "_tokens"])


def native_cases():
    z = load_golden("native")
    return sorted({k.split("/")[0] for k in z.files})


def native_case(z, name):
    p = {k[len(name) + 7:]: z[k].astype(np.float64) for k in z.files if k.startswith(name + "/param/")}
    train, fused, ln, prefix, stack, carry = [int(v) for v in z[name + "/cfg"]]
    kw = dict(L=2, D=16, train=bool(train), fused=bool(fused), ln=bool(ln),
              decay_mode="prefix_sum" if prefix else "learned", stack=stack, lambda_decay=0.05)
    if carry:
        kw.update(h0=z[name + "/h0"], s0=z[name + "/s0"])
    return p, kw


@pytest.mark.parametrize("name", native_cases())
def test_native_lucyrnn_oracle_vs_reference(name):
    """oracle/native.py == reference lucyrnn.LucyRNN (train quirks of SURVEY F9 included)."""
    from oracle import native
    z = load_golden("native")
    p, kw = native_case(z, name)
    logits, h, s = native.lucyrnn_forward(p, z[name + "/x"], **kw)
    np.testing.assert_allclose(logits, z[name + "/logits"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(np.stack(h), z[name + "/h"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(np.stack(s), z[name + "/s"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("T,U", [(1, 0), (1, 2), (2, 0), (3, 2), (4, 3), (2, 4)])
def test_rnnt_oracle_vs_brute_force_alignments(T, U):
    """RNN-T parity is unpinned against warp_rnnt (absent): the lattice restatement
    is pinned against the definition, -log of the sum over every monotonic alignment."""
    from oracle import rnnt
    rng = np.random.default_rng(10 * T + U)
    x = rng.standard_normal((T, U + 1, 5))
    lp = x - np.log(np.exp(x).sum(-1, keepdims=True))
    y = rng.integers(1, 5, U)
    nll, g = rnnt.rnnt_single(lp, y)
    np.testing.assert_allclose(nll, rnnt.brute_force_nll(lp, y), rtol=1e-12)
    # gradient: central differences of the lattice nll
    eps = 1e-6
    for idx in [(0, 0, 0), (T - 1, U, 0)] + ([(0, 0, int(y[0]))] if U else []):
        d = np.zeros_like(lp)
        d[idx] = eps
        fd = (rnnt.rnnt_single(lp + d, y)[0] - rnnt.rnnt_single(lp - d, y)[0]) / (2 * eps)
        np.testing.assert_allclose(g[idx], fd, rtol=1e-6, atol=1e-9)
    # occupancies: every alignment spends exactly one blank per frame and emits all U labels
    np.testing.assert_allclose(g[:, :, 0].sum(axis=1), -1.0, rtol=1e-10)
    np.testing.assert_allclose(g[:, :, 1:].sum(), -float(U), rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("name", ["small", "state", "c4"])
def test_mlstm_oracle_vs_hf_chunkwise(name):
    """oracle/mlstm.py (step recurrence) == HF transformers' chunkwise mLSTM (fixture)."""
    from oracle import mlstm
    z = load_golden("mlstm")
    g = lambda k: z.get(f"{name}/{k}") if f"{name}/{k}" in z.files else None  # noqa: E731
    h, (C, n, m) = mlstm.mlstm_recurrent(g("q"), g("k"), g("v"), g("igate"), g("fgate"),
                                         g("c0"), g("n0"), g("m0"))
    np.testing.assert_allclose(h, g("h"), rtol=2e-4, atol=2e-5 * np.abs(g("h")).max())
    np.testing.assert_allclose(C, g("cT"), rtol=2e-4, atol=2e-5 * np.abs(g("cT")).max())
    np.testing.assert_allclose(n, g("nT"), rtol=2e-4, atol=2e-5 * np.abs(g("nT")).max())
    np.testing.assert_allclose(m, g("mT"), rtol=1e-5, atol=1e-5)


def test_fbank_oracle_vs_independent_restatement():
    """oracle/fbank.py (torchaudio's MFCC / MelSpectrogram+AmplitudeToDB as make_frontend builds
    them, model.py:250-279) against tests/golden/fbank.npz, produced by transformers'
    audio_utils spectrogram / mel_filter_bank / power_to_db and scipy's orthonormal DCT
    (tests/golden/gen_fbank.py); parity w.r.t. torchaudio itself is unpinned (absent)."""
    from oracle import fbank as ofb
    z = load_golden("fbank")
    a = z["audio"]
    p = ofb.power_spectrogram(a)
    np.testing.assert_allclose(p, z["power"], rtol=1e-5, atol=1e-6 * np.abs(z["power"]).max())
    np.testing.assert_allclose(p @ ofb.melscale_fbanks(), z["mel"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(ofb.frontend(a, "mfcc"), z["mfcc"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(ofb.frontend(a, "mel"), z["logmel_db"], rtol=1e-5, atol=1e-4)
    assert ofb.frontend(a[:, :399], "mfcc").shape == (3, 0, 80)


MODULE_CASES = ["d64_init", "d64_proj", "d40_proj"]


def module_params(z, name):
    """module.npz's reference state_dict -> oracle.lucy_step parameter names."""
    pre = name + "/param/"
    L = len([k for k in z.files if k.startswith(pre + "tracks.0.") and k.endswith(".linear.weight")])
    p = {}
    for l in range(L):
        p[f"W{l}"] = z[pre + f"tracks.0.{l}.linear.weight"]
        p[f"b{l}"] = z[pre + f"tracks.0.{l}.linear.bias"]
        if l < L - 1:
            p[f"g{l}"] = z[pre + f"norms.0.{l}.weight"]
            p[f"be{l}"] = z[pre + f"norms.0.{l}.bias"]
    p["Wo"] = z[pre + "output_proj.weight"]
    p["bo"] = z[pre + "output_proj.bias"]
    return p, L, p["W0"].shape[0] // 7


@pytest.mark.parametrize("name", MODULE_CASES)
def test_lucy_step_forward_vs_reference_module(name):
    """oracle.lucy_step.forward against the reference LucyRNNtriton itself (Triton interpreter,
    fp32, its own init, 3 layers + LayerNorms + output_proj, two segments with state carry);
    tolerance: tests.conftest.assert_ref_parity (the reference's own fp32-vs-fp64 noise)."""
    from oracle import lucy_step
    from tests.conftest import assert_ref_parity
    z = load_golden("module")
    p, L, D = module_params(z, name)
    state = None
    for seg in range(2):
        logits, (h, s), _, _ = lucy_step.forward(p, z[f"{name}/seg{seg}/x"], L, D, state)
        pre = f"{name}/seg{seg}/"
        assert_ref_parity(logits, z[pre + "logits"], z[pre + "logits64"])
        assert_ref_parity(np.stack(h), z[pre + "h"], z[pre + "h64"])
        assert_ref_parity(np.stack(s), z[pre + "s"], z[pre + "s64"])
        state = (h, s)


@pytest.mark.parametrize("T,U", [(1, 0), (4, 0), (1, 3), (7, 5), (23, 11)])
def test_rnnt_vectorised_lattice_vs_loop_oracle(T, U):
    """oracle.lucy_step.rnnt_lattice (anti-diagonal form, used by the C5 step oracle) against
    oracle.rnnt.rnnt_single (pinned by brute-force alignment sums)."""
    from oracle import lucy_step, rnnt
    rng = np.random.default_rng(T * 31 + U)
    V = 9
    lp = torch.from_numpy(rng.standard_normal((T, U + 1, V))).log_softmax(-1).numpy()
    y = rng.integers(1, V, U)
    nll_ref, g = rnnt.rnnt_single(lp, y, 0)
    nll, gb, gy = lucy_step.rnnt_lattice(lp[:, :, 0], lp[:, np.arange(U), y] if U else np.zeros((T, 0)))
    np.testing.assert_allclose(nll, nll_ref, rtol=1e-12)
    np.testing.assert_allclose(gb, g[:, :, 0], atol=1e-12)
    for u in range(U):
        gref = g[:, u, y[u]] - (g[:, u, 0] if y[u] == 0 else 0)
        np.testing.assert_allclose(gy[:, u], gref, atol=1e-12)


@pytest.mark.parametrize("round_bf16", [False, True])
def test_rnnt_joint_oracle_grads_vs_autograd(round_bf16):
    """oracle.lucy_step.rnnt_joint_loss_grad (the C5 joiner + lattice oracle) against torch
    autograd through the same joint in fp64 with the lattice gradient injected at the log-probs
    (the lattice itself is pinned above): ragged lengths, U = 0 included."""
    from oracle import lucy_step, rnnt
    rng = np.random.default_rng(5)
    B, T, U, J, V = 3, 11, 4, 8, 12
    enc_p = rng.standard_normal((B, T, J))
    pred_p = rng.standard_normal((B, U + 1, J))
    W = rng.standard_normal((V, J)).astype(np.float32)
    bias = rng.standard_normal(V)
    labels = rng.integers(1, V, (B, U))
    fl, ll = [11, 6, 9], [4, 2, 0]
    nll, de, dp, dW, db = lucy_step.rnnt_joint_loss_grad(enc_p, pred_p, W, bias, labels, fl, ll, 0,
                                                         round_bf16=round_bf16, t_chunk=4)
    e = torch.tensor(enc_p, requires_grad=True)
    pp = torch.tensor(pred_p, requires_grad=True)
    w = torch.tensor(W.astype(np.float64), requires_grad=True)
    b = torch.tensor(bias, requires_grad=True)
    z = torch.tanh(e.unsqueeze(2) + pp.unsqueeze(1))
    if round_bf16:
        z = z + (z.to(torch.bfloat16).double() - z).detach()
        w = w + (w.to(torch.bfloat16).double() - w).detach()
    lp = (z @ w.t() + b).log_softmax(-1)
    glp = torch.zeros_like(lp)
    ref = []
    for i in range(B):
        n, g = rnnt.rnnt_single(lp[i, :fl[i], :ll[i] + 1].detach().numpy(), labels[i, :ll[i]], 0)
        ref.append(n)
        glp[i, :fl[i], :ll[i] + 1] = torch.from_numpy(g)
    lp.backward(glp)
    np.testing.assert_allclose(nll, ref, rtol=1e-12)
    wg = w.grad if not round_bf16 else None
    for got, r in [(de, e.grad), (dp, pp.grad), (db, b.grad)] + ([(dW, wg)] if wg is not None else []):
        np.testing.assert_allclose(got, r.numpy(), rtol=1e-9, atol=1e-12)
