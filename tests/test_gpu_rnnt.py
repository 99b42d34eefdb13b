"""GPU parity of the RNN-T loss kernels (rnnt.hip) against oracle/rnnt.py (fp64 lattice, itself
pinned against brute-force alignment sums; warp_rnnt parity is unpinned — SURVEY §8c).
Tolerances: nll 1e-5 relative (fp32 lattice with fp64 offsets); gradients 1e-4 relative to the
tensor's max (fp32 rows), bf16 logits 1e-2."""
import numpy as np
import pytest
import torch

from oracle import rnnt as ornnt

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def ops():
    from statecatcher_amd import ops as o
    return o


def make(B, T, U, V, seed, ragged=True):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, T, U + 1, V)).astype(np.float32) * 1.5
    labels = rng.integers(1, V, (B, max(U, 1)))
    fl = np.full(B, T) if not ragged else rng.integers(max(1, T // 2), T + 1, B)
    ll = np.full(B, U) if not ragged else rng.integers(0, U + 1, B)
    fl[0], ll[0] = T, U
    return x, labels, fl, ll


def ref(x, labels, fl, ll, logits, reduction="mean", average_frames=False):
    lp = x - np.log(np.exp(x.astype(np.float64)).sum(-1, keepdims=True)) if logits else x
    loss, costs, g = ornnt.rnnt_loss(lp, labels, fl, ll, reduction=reduction,
                                     average_frames=average_frames)
    if logits and g is not None:   # chain rule through log_softmax
        sm = np.exp(lp)
        g = g - sm * g.sum(-1, keepdims=True)
    return loss, costs, g


# U + 1 <= 64, 128, 192, 256 (the opt-in one-wave lattice's 1, 2, 3, 4 label positions per lane
# when SC_RNNT_AB1=1), then the multi-wave one's largest case (15 waves, K = 8)
DENSE_CASES = [(3, 7, 4, 11), (2, 1, 3, 5), (2, 9, 0, 6), (4, 40, 12, 33), (2, 130, 70, 17),
               (2, 60, 150, 9), (2, 30, 220, 7), (2, 24, 800, 5)]


@pytest.mark.parametrize("B,T,U,V", DENSE_CASES)
@pytest.mark.parametrize("logits", [True, False])
def test_rnnt_dense_vs_oracle(B, T, U, V, logits):
    _dense_check(B, T, U, V, logits)


def test_rnnt_one_wave_lattice_vs_oracle():
    """The opt-in one-wave lattice (rnnt_ab1_kernel, SC_RNNT_AB1=1, read once per process, so it
    runs in a child process): every DENSE_CASES lattice with U + 1 <= 256 takes it (1 .. 4
    label positions per lane, its kh = kAb1R / 2 offset indexing and terminal blank), the last
    one falls back to the multi-wave kernel; nll, costs and gradients vs the oracle as above."""
    import os
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, '.'); from tests.test_gpu_rnnt import DENSE_CASES, "
            "_dense_check\nfor c in DENSE_CASES:\n  for lg in (True, False): _dense_check(*c, lg)\n"
            "print('ONE-WAVE OK')")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, "-c", code], cwd=root, env=dict(os.environ, SC_RNNT_AB1="1"),
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0 and "ONE-WAVE OK" in p.stdout, p.stderr[-3000:]


def _dense_check(B, T, U, V, logits):
    x, labels, fl, ll = make(B, T, U, V, seed=B * 100 + T + U)
    if not logits:
        x = x - np.log(np.exp(x).sum(-1, keepdims=True))
    xt = torch.as_tensor(x).to(DEV).requires_grad_(True)
    loss = ops().rnnt_loss(xt, torch.as_tensor(labels).to(DEV), torch.as_tensor(fl).to(DEV),
                           torch.as_tensor(ll).to(DEV), is_logits=logits)
    loss.backward()
    rl, costs, rg = ref(x, labels, fl, ll, logits)
    np.testing.assert_allclose(loss.item(), rl, rtol=1e-5)
    g = xt.grad.cpu().numpy()
    np.testing.assert_allclose(g, rg, rtol=1e-4, atol=1e-4 * np.abs(rg).max())
    nll = ops().rnnt_loss(xt.detach(), torch.as_tensor(labels).to(DEV), torch.as_tensor(fl).to(DEV),
                          torch.as_tensor(ll).to(DEV), reduction="none", is_logits=logits)
    np.testing.assert_allclose(nll.cpu().numpy(), costs, rtol=1e-5)


def test_rnnt_compact_layout_equals_dense():
    B, T, U, V = 3, 11, 5, 9
    x, labels, fl, ll = make(B, T, U, V, seed=4)
    rows = np.concatenate([x[b, :fl[b], :ll[b] + 1].reshape(-1, V) for b in range(B)])
    xc = torch.as_tensor(rows).to(DEV).requires_grad_(True)
    args = (torch.as_tensor(labels).to(DEV), torch.as_tensor(fl).to(DEV), torch.as_tensor(ll).to(DEV))
    lc = ops().rnnt_loss(xc, *args, compact=True, is_logits=True, reduction="sum")
    lc.backward()
    rl, _, rg = ref(x, labels, fl, ll, True, reduction="sum")
    np.testing.assert_allclose(lc.item(), rl, rtol=1e-5)
    rgc = np.concatenate([rg[b, :fl[b], :ll[b] + 1].reshape(-1, V) for b in range(B)])
    np.testing.assert_allclose(xc.grad.cpu().numpy(), rgc, rtol=1e-4, atol=1e-4 * np.abs(rgc).max())


def test_rnnt_long_lattice_bf16_logits_and_determinism():
    """T=1500, U=150 (config C5's lattice) with bf16 logits: loss vs the fp64 oracle on the same
    rounded inputs, bitwise-deterministic gradients."""
    B, T, U, V = 2, 1500, 150, 8
    x, labels, fl, ll = make(B, T, U, V, seed=9, ragged=False)
    xb = torch.as_tensor(x).bfloat16()
    xt = xb.to(DEV).requires_grad_(True)
    args = (torch.as_tensor(labels).to(DEV), torch.as_tensor(fl).to(DEV), torch.as_tensor(ll).to(DEV))
    grads = []
    for _ in range(2):
        xt.grad = None
        loss = ops().rnnt_loss(xt, *args, is_logits=True)
        loss.backward()
        grads.append(xt.grad.clone())
    assert torch.equal(grads[0], grads[1])
    rl, _, rg = ref(xb.float().numpy(), labels, fl, ll, True)
    np.testing.assert_allclose(loss.item(), rl, rtol=1e-5)
    g = grads[0].float().cpu().numpy()
    np.testing.assert_allclose(g, rg, rtol=2e-2, atol=1e-2 * np.abs(rg).max())


def test_rnnt_compute_loss_with_joiner_matches_reference_sequence():
    """compute_loss('rnnt') with the fused RNNTLoss == the reference sequence (joiner ->
    log_softmax fp32 -> loss) evaluated with the oracle, gradients through the joiner."""
    import statecatcher_amd as sc
    torch.manual_seed(3)
    B, T, Din, V, U = 2, 12, 10, 7, 4
    joiner = sc.RNNTPredictorJoiner(enc_out_dim=V, pred_emb_dim=6, join_dim=8, vocab_size=V).to(DEV)

    class Enc(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(Din, V)

        def forward(self, feats, mask, states=None):
            return self.lin(feats), None
    enc = Enc().to(DEV)
    feats = torch.randn(B, T, Din, device=DEV)
    tokens = torch.randint(1, V, (B, U), device=DEV)
    loss, _, _, _ = sc.compute_loss("rnnt", sc.RNNTLoss(), enc, feats, None, tokens, [T, T - 3],
                                    [U, U - 1], 0, use_rnnt_joiner=joiner)
    loss.backward()
    with torch.no_grad():
        logits = joiner(enc(feats, None)[0], torch.cat([torch.zeros(B, 1, dtype=tokens.dtype,
                                                                    device=DEV), tokens], 1))
    lp = logits.double().log_softmax(-1).cpu().numpy()
    rl, _, _ = ornnt.rnnt_loss(lp, tokens.cpu().numpy(), [T, T - 3], [U, U - 1])
    np.testing.assert_allclose(loss.item(), rl, rtol=1e-5)
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in joiner.parameters())


def test_rnnt_zero_frames_is_infinite():
    x = torch.randn(2, 3, 2, 4, device=DEV)
    nll = ops().rnnt_loss(x, torch.ones(2, 1, dtype=torch.int64, device=DEV),
                          torch.tensor([0, 3], device=DEV), torch.tensor([1, 1], device=DEV),
                          reduction="none", is_logits=True)
    assert torch.isinf(nll[0]) and torch.isfinite(nll[1])
