"""GPU parity of the mLSTM cell kernels (mlstm.hip).  The kernels compute in bf16/f16 (the
reference runs its kernels under autocast_kernel_dtype=float16) with fp32 state, so the
checkers are evaluated in fp64 on the SAME rounded inputs: oracle/mlstm.py (forward) and its
torch restatement tests/torch_ref.mlstm64 (gradients), both pinned to HF transformers'
chunkwise mLSTM by tests/test_oracle_golden.py / tests/golden/mlstm.npz.  Rows whose
normaliser q.n nearly cancels amplify the unavoidable bf16 rounding of the intermediate tiles,
so tensors are compared by relative Frobenius error (<= 1e-2 outputs, <= 3e-2 gradients) and
elementwise at 10% of the tensor's scale.  Parity against the reference's own xLSTM fork is
unpinned."""
import numpy as np
import pytest
import torch

from oracle import mlstm as omlstm
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def ops():
    from statecatcher_amd import ops as o
    return o


def close(got, ref, frac):
    got = got.detach().double().cpu().numpy() if isinstance(got, torch.Tensor) else got
    ref = ref.detach().double().cpu().numpy() if isinstance(ref, torch.Tensor) else np.asarray(ref)
    scale = max(float(np.abs(ref).max()), 1e-30)
    rel = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30)
    assert rel <= frac, f"relative Frobenius error {rel:.3e} > {frac}"
    np.testing.assert_allclose(got, ref, rtol=0.1, atol=0.1 * scale)


@pytest.mark.parametrize("name", ["small", "state", "c4"])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_mlstm_fwd_bwd_vs_fp64_on_rounded_inputs(name, dtype):
    from tests.torch_ref import mlstm64
    z = load_golden("mlstm")
    g = lambda k: torch.as_tensor(z[f"{name}/{k}"]) if f"{name}/{k}" in z.files else None  # noqa
    ins = {key: g(key).to(dtype) for key in ("q", "k", "v")}
    ins.update({key: g(key) for key in ("igate", "fgate", "c0", "n0") if g(key) is not None})
    m0 = g("m0")
    leaves = {key: t.to(DEV).requires_grad_(True) for key, t in ins.items()}
    h, (cT, nT, mT) = ops().mlstm_chunkwise(leaves["q"], leaves["k"], leaves["v"], leaves["igate"],
                                           leaves["fgate"], leaves.get("c0"), leaves.get("n0"),
                                           None if m0 is None else m0.to(DEV),
                                           return_last_states=True)
    ref_leaves = {key: t.double().requires_grad_(True) for key, t in ins.items()}
    rh, (rc, rn, rm) = mlstm64(ref_leaves["q"], ref_leaves["k"], ref_leaves["v"], ref_leaves["igate"],
                               ref_leaves["fgate"], ref_leaves.get("c0"), ref_leaves.get("n0"),
                               None if m0 is None else m0.double())
    close(h, rh, 1e-2)
    close(cT, rc, 1e-2)
    close(nT, rn, 1e-2)
    np.testing.assert_allclose(mT.cpu().numpy(), rm.detach().numpy(), rtol=1e-5, atol=1e-5)
    R = g("R")
    (h.float() * R.to(DEV)).sum().backward()
    (rh * R.double()).sum().backward()
    for key, t in leaves.items():
        close(t.grad, ref_leaves[key].grad, 3e-2)


def test_mlstm_fp32_reference_fixture_at_bf16_tolerance():
    """Against HF's own fp64 outputs on the unrounded inputs (the fixture itself)."""
    z = load_golden("mlstm")
    h = ops().mlstm_chunkwise(*[torch.as_tensor(z[f"c4/{k}"]).to(DEV)
                                for k in ("q", "k", "v", "igate", "fgate", "c0", "n0", "m0")])
    close(h, z["c4/h"], 3e-2)


def test_mlstm_fp32_inputs_run_the_f16_cell():
    """fp32 q / k / v (an fp32 xLSTM without autocast) go through the f16 cell, the finer of the
    two compiled cells: bitwise the explicit f16 call, and against fp64 on the
    UNROUNDED inputs closer than the bf16 cell gets (f16 rounding is 8x finer)."""
    from tests.torch_ref import mlstm64
    z = load_golden("mlstm")
    ins = [torch.as_tensor(z[f"c4/{k}"]) for k in ("q", "k", "v", "igate", "fgate")]
    R = torch.as_tensor(z["c4/R"]) if "c4/R" in z.files else torch.randn_like(ins[2])
    errs = {}
    for dt in (torch.float32, torch.float16, torch.bfloat16):
        leaves = [t.to(DEV).to(dt if i < 3 else torch.float32).requires_grad_(True)
                  for i, t in enumerate(ins)]
        h = ops().mlstm_chunkwise(*leaves)
        (h.float() * R.to(DEV)).sum().backward()
        errs[dt] = (h.detach().float(), [t.grad.float() for t in leaves])
    assert torch.equal(errs[torch.float32][0], errs[torch.float16][0])
    for a, b in zip(errs[torch.float32][1], errs[torch.float16][1]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-6)   # fp32 vs f16 gradient casts only
    ref = [t.double().requires_grad_(True) for t in ins]
    rh, _ = mlstm64(*ref)
    (rh * R.double()).sum().backward()

    def rel(a, b):
        return float((a.double().cpu() - b).norm() / b.norm())
    e32 = [rel(errs[torch.float32][0], rh.detach())] + \
        [rel(g, r.grad) for g, r in zip(errs[torch.float32][1], ref)]
    ebf = [rel(errs[torch.bfloat16][0], rh.detach())] + \
        [rel(g, r.grad) for g, r in zip(errs[torch.bfloat16][1], ref)]
    print("fp32-input (f16 cell) vs fp64:", [f"{e:.2e}" for e in e32],
          "bf16 cell:", [f"{e:.2e}" for e in ebf])
    assert e32[0] <= 5e-3 and max(e32) <= 2e-2, e32
    assert e32[0] < ebf[0] and e32[1] < ebf[1], (e32, ebf)


def test_mlstm_fp32_inputs_beyond_f16_range_run_the_bf16_cell():
    """fp32 q / k / v with a value above f16's 65504: the f16 cell would turn it into
    inf and the outputs into NaN; the fp32 path then takes the bf16 cell (fp32's range) and is
    bitwise the explicit bf16 call, finite, in the forward and the backward."""
    z = load_golden("mlstm")
    ins = [torch.as_tensor(z[f"c4/{k}"]) for k in ("q", "k", "v", "igate", "fgate")]
    ins[2] = ins[2].clone()
    ins[2][0, 0, 5, 3] = 1.0e5   # one v element past f16's range
    outs = {}
    for dt in (torch.float32, torch.bfloat16):
        leaves = [t.to(DEV).to(dt if i < 3 else torch.float32).requires_grad_(True)
                  for i, t in enumerate(ins)]
        h = ops().mlstm_chunkwise(*leaves)
        h.float().sum().backward()
        outs[dt] = (h.detach().float(), [t.grad.float() for t in leaves])
    assert torch.isfinite(outs[torch.float32][0]).all()
    assert torch.equal(outs[torch.float32][0], outs[torch.bfloat16][0])
    for a, b in zip(outs[torch.float32][1], outs[torch.bfloat16][1]):
        assert torch.isfinite(a).all()
        torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-6)   # fp32 vs bf16 gradient casts only


def test_mlstm_long_sequence_vs_oracle_and_state_carry():
    """T = 1536 (the C4 segment after padding to 64): h and final state vs the numpy step
    recurrence; two carried halves equal one pass."""
    torch.manual_seed(0)
    B, NH, T, DQ, DV = 1, 2, 1536, 64, 128
    q, k = torch.randn(B, NH, T, DQ), torch.randn(B, NH, T, DQ)
    v = torch.randn(B, NH, T, DV)
    ig, fg = torch.randn(B, NH, T) * 3, torch.randn(B, NH, T) * 2 + 3
    qb, kb, vb = (x.bfloat16() for x in (q, k, v))
    args = [x.to(DEV) for x in (qb, kb, vb, ig, fg)]
    h, (C, n, m) = ops().mlstm_chunkwise(*args, return_last_states=True)
    rh, (rC, rn, rm) = omlstm.mlstm_recurrent(qb.float().numpy(), kb.float().numpy(),
                                              vb.float().numpy(), ig.numpy(), fg.numpy())
    close(h, rh, 2e-2)
    close(C, rC, 2e-2)
    np.testing.assert_allclose(m.cpu().numpy(), rm, rtol=1e-4, atol=1e-4)
    half = T // 2
    h1, st = ops().mlstm_chunkwise(*[a[:, :, :half] for a in args], return_last_states=True)
    h2, (C2, _, _) = ops().mlstm_chunkwise(*[a[:, :, half:] for a in args], *st,
                                           return_last_states=True)
    torch.testing.assert_close(torch.cat([h1, h2], 2).float(), h.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(C2, C, rtol=1e-3, atol=1e-3)


def test_mlstm_rejects_unsupported_shapes():
    q = torch.randn(1, 1, 100, 64, device=DEV, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        ops().mlstm_chunkwise(q, q, torch.randn(1, 1, 100, 128, device=DEV, dtype=torch.bfloat16),
                              torch.zeros(1, 1, 100, device=DEV), torch.zeros(1, 1, 100, device=DEV))


def test_xlstm_block_vs_hf_block_fixture():
    """statecatcher_amd.xlstm.xLSTMBlock with the HF block's weights reproduces HF's fp64 block
    (mLSTM layer + FFN, RMSNorms, multi-head LayerNorm, soft-capped gates): output, final state,
    and gradients w.r.t. the input, a projection weight and a gate bias (bf16 cell)."""
    from statecatcher_amd.xlstm import xLSTMBlock, xLSTMLargeConfig
    z = load_golden("mlstm")
    cfg = xLSTMLargeConfig(embedding_dim=128, num_heads=2, num_blocks=1, vocab_size=10)
    blk = xLSTMBlock(cfg)
    blk.load_state_dict({k[len("block/param/"):]: torch.as_tensor(z[k]) for k in z.files
                         if k.startswith("block/param/")})
    blk = blk.to(DEV)
    x = torch.as_tensor(z["block/x"]).to(DEV).requires_grad_(True)
    y, (c, n, m) = blk(x)
    close(y, z["block/y"], 1e-2)
    close(c, z["block/cT"], 2e-2)
    (y * torch.as_tensor(z["block/R"]).to(DEV)).sum().backward()
    close(x.grad, z["block/dx"], 3e-2)
    close(blk.mlstm_layer.q.weight.grad, z["block/dq_weight"], 3e-2)
    # the forget-gate bias gradient sums reverse cumulative differences q.dq - k.dk over every
    # step: it carries the bf16 rounding of the whole cell input (HF ran fp64 on fp32 inputs)
    close(blk.mlstm_layer.fgate_preact.bias.grad, z["block/dfgate_bias"], 5e-2)


def test_xlstm_asr_ctc_training_step_runs_and_learns():
    """ASRModel(xLSTM) + fused CTC through SegmentTrainer: T padded to 64 with the mask, state
    dict carried across segments, loss decreases on a fixed batch."""
    import statecatcher_amd as sc
    from statecatcher_amd.model import build_xlstm_config
    from statecatcher_amd.train import SegmentTrainer
    torch.manual_seed(0)
    B, T, F, V = 2, 150, 80, 24
    model = sc.ASRModel(None, build_xlstm_config(F, V, num_heads=2, num_blocks=2, embedding_dim=128),
                        V, F, -1).to(DEV)
    opt = torch.optim.Adam(model.parameters(), lr=2e-3)
    tr = SegmentTrainer(model, sc.CTCLoss(), opt, amp_dtype=torch.bfloat16)
    feats = torch.randn(B, T, F, device=DEV)
    masks = torch.ones(B, T, dtype=torch.bool, device=DEV)
    tok = torch.randint(1, V, (B, 10), device=DEV)
    losses = []
    for it in range(25):
        if it % 5 == 0:
            tr.begin_batch()
        losses.append(float(tr.train_segment(feats, masks, tok, [T] * B, [10] * B).detach()))
    assert isinstance(tr.encoder_state, dict) and len(tr.encoder_state) == 2
    assert np.isfinite(losses).all()
    assert np.mean(losses[-3:]) < 0.8 * np.mean(losses[:3])


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("DQ,DV,T", [(96, 192, 320), (32, 64, 192), (64, 128, 128)])
def test_mlstm_fwd_split_bitwise_equals_walk(dtype, DQ, DV, T, monkeypatch):
    """The forward as a state walk + chunk-parallel output kernel (default) is bitwise the single
    walk (SC_MLSTM_SPLIT=0): same operations on the same state image, so h, the carried state
    and every gradient (the backward reads the forward's state image, m and den) agree exactly,
    with and without an initial state."""
    g = torch.Generator(device=DEV).manual_seed(7)
    BH = 6
    q = torch.randn(1, BH, T, DQ, device=DEV, generator=g).to(dtype)
    k = torch.randn(1, BH, T, DQ, device=DEV, generator=g).to(dtype)
    v = torch.randn(1, BH, T, DV, device=DEV, generator=g).to(dtype)
    ig = torch.randn(1, BH, T, device=DEV, generator=g) * 3
    fg = torch.randn(1, BH, T, device=DEV, generator=g) * 2 + 3
    c0 = torch.randn(1, BH, DQ, DV, device=DEV, generator=g) * 0.1
    n0 = torch.randn(1, BH, DQ, device=DEV, generator=g) * 0.1
    m0 = torch.randn(1, BH, 1, device=DEV, generator=g)
    dh = torch.randn(1, BH, T, DV, device=DEV, generator=g).to(dtype)

    def run(split, init):
        monkeypatch.setenv("SC_MLSTM_SPLIT", "1" if split else "0")
        leaves = [x.clone().requires_grad_(True) for x in (q, k, v, ig, fg)]
        st = (c0, n0, m0) if init else (None, None, None)
        h, (C, n, m) = ops().mlstm_chunkwise(*leaves, *st, return_last_states=True)
        torch.autograd.backward([h, C.sum()], [dh, None])
        torch.cuda.synchronize()
        return [h, C, n, m] + [x.grad for x in leaves]

    for init in (False, True):
        a, b = run(True, init), run(False, init)
        for i, (x, y) in enumerate(zip(a, b)):
            assert torch.equal(x, y), (init, i)
