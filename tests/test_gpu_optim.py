"""GPU parity of the optimizer-side HIP kernels (csrc/optim.hip) against torch itself:

* ``optim.clip_and_adam_step`` vs ``torch.nn.utils.clip_grad_norm_`` + ``torch.optim.Adam`` /
  ``AdamW`` single-tensor steps (the reference's train.py:543-552 / :112-136).  Same fp32
  formulas and the same scalar roundings (Python doubles cast once to float); the remaining
  differences are the norm's summation order (fp64 here) and FMA contraction: parameters and
  moments within 2e-6 relative, the returned norm within 1e-5.
* ``ops.weight_images`` vs ``w.to(bf16)`` (+ step-blocked row permutation, zero pad columns,
  transpose): bit-exact (both round to nearest even).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def _params(seed, shapes, unaligned=False):
    g = torch.Generator(device=DEV).manual_seed(seed)
    ps = []
    for sh in shapes:
        n = 1
        for d in sh:
            n *= d
        if unaligned:   # a parameter whose data starts 4 bytes into its storage (scalar path)
            base = torch.randn(n + 1, device=DEV, generator=g)
            ps.append(torch.nn.Parameter(base[1:].view(sh)))
        else:
            ps.append(torch.nn.Parameter(torch.randn(*sh, device=DEV, generator=g)))
    return ps


def _twin(ps):
    return [torch.nn.Parameter(p.detach().clone()) for p in ps]


def _set_grads(ps, qs, seed, scale):
    g = torch.Generator(device=DEV).manual_seed(seed)
    for p, q in zip(ps, qs):
        gr = torch.randn(p.shape, device=DEV, generator=g) * scale
        p.grad = gr.clone()
        q.grad = gr.clone()


def _close(a, b, rtol=2e-6, atol=1e-7):
    torch.testing.assert_close(a, b, rtol=rtol, atol=atol)


SHAPES = [(3584, 512), (1024,), (7,), (5, 13), (3, 1), (1024, 512)]


@pytest.mark.parametrize("kind,kw", [
    ("adam", {}),
    ("adam", {"weight_decay": 0.01, "betas": (0.9, 0.98), "eps": 1e-6}),
    ("adamw", {"weight_decay": 0.05}),
    # torch.optim.Adam with AdamW's update (a per-group flag since torch 2.6)
    ("adam", {"weight_decay": 0.05, "decoupled_weight_decay": True}),
])
@pytest.mark.parametrize("unaligned", [False, True])
def test_clip_adam_matches_torch(kind, kw, unaligned):
    from statecatcher_amd.optim import clip_and_adam_step, hip_adam_eligible
    cls = torch.optim.Adam if kind == "adam" else torch.optim.AdamW
    ps = _params(1, SHAPES, unaligned)
    qs = _twin(ps)
    ours = cls(ps, lr=3e-3, **kw)
    ref = cls(qs, lr=3e-3, foreach=False, **kw)
    assert hip_adam_eligible(ours)
    # steps that clip (norm >> 50), that do not (norm < 50), and clip again
    for k, scale in enumerate([3.0, 0.01, 1.0, 0.02]):
        _set_grads(ps, qs, 10 + k, scale)
        n_ours = clip_and_adam_step(ours, ps, 50.0)
        n_ref = torch.nn.utils.clip_grad_norm_(qs, 50.0)
        ref.step()
        _close(n_ours, n_ref, rtol=1e-5, atol=0)
        for p, q in zip(ps, qs):
            _close(p, q)
            so, sr = ours.state[p], ref.state[q]
            assert float(so["step"]) == float(sr["step"]) == k + 1
            assert so["step"].device.type == "cpu"
            _close(so["exp_avg"], sr["exp_avg"])
            _close(so["exp_avg_sq"], sr["exp_avg_sq"], rtol=2e-6, atol=1e-12)


def test_clip_scope_and_missing_grads():
    """Parameters outside the clip set step unclipped (an RNN-T joiner next to the model: the
    reference clips model.parameters() only); parameters without a gradient are skipped and
    keep their step count."""
    from statecatcher_amd.optim import clip_and_adam_step
    ps = _params(2, [(512, 64), (64,), (33,), (8, 8)])
    qs = _twin(ps)
    ours = torch.optim.Adam(ps, lr=1e-3)
    ref = torch.optim.Adam(qs, lr=1e-3, foreach=False)
    _set_grads(ps, qs, 3, 5.0)
    ps[3].grad = None
    qs[3].grad = None
    clip_and_adam_step(ours, ps[:2], 1.0)
    torch.nn.utils.clip_grad_norm_(qs[:2], 1.0)
    ref.step()
    for p, q in zip(ps, qs):
        _close(p, q)
    assert ps[3] not in ours.state or not ours.state[ps[3]]


def test_state_dict_interop():
    """HIP steps leave torch's own optimizer state: a torch Adam loaded from it continues
    identically, and vice versa."""
    from statecatcher_amd.optim import clip_and_adam_step
    ps = _params(4, [(256, 128), (128,)])
    qs = _twin(ps)
    ours = torch.optim.Adam(ps, lr=2e-3)
    ref = torch.optim.Adam(qs, lr=2e-3, foreach=False)
    for k in range(2):
        _set_grads(ps, qs, 20 + k, 1.0)
        clip_and_adam_step(ours, ps, 10.0)
        torch.nn.utils.clip_grad_norm_(qs, 10.0)
        ref.step()
    ref2 = torch.optim.Adam(qs, lr=2e-3, foreach=False)
    import copy
    ref2.load_state_dict(copy.deepcopy(ours.state_dict()))   # (load_state_dict aliases tensors)
    _set_grads(ps, qs, 30, 1.0)
    ref2.step()
    ours.step()   # torch's own step on the state the HIP path built
    for p, q in zip(ps, qs):
        _close(p, q)


def test_ineligible_optimizers():
    from statecatcher_amd.optim import clip_and_adam_step, hip_adam_eligible
    ps = _params(5, [(16,)])
    assert not hip_adam_eligible(torch.optim.Adam(ps, lr=1e-3, amsgrad=True))
    assert not hip_adam_eligible(torch.optim.Adam(ps, lr=1e-3, fused=True))
    assert not hip_adam_eligible(torch.optim.SGD(ps, lr=1e-3))
    cpu = [torch.nn.Parameter(torch.zeros(4))]
    assert not hip_adam_eligible(torch.optim.Adam(cpu, lr=1e-3))
    with pytest.raises(RuntimeError):
        clip_and_adam_step(torch.optim.SGD(ps, lr=1e-3), ps, 1.0)


@pytest.mark.parametrize("max_norm", [50.0, 1e-3])
def test_trainer_step_uses_hip_adam(max_norm, monkeypatch):
    """SegmentTrainer with the reference's optim.Adam(params, lr) (train.py:133) steps through
    clip_and_adam_step and equals clip_grad_norm_ (train.py:553) + torch's single-tensor Adam,
    with the clip inactive (50) and active (1e-3)."""
    import copy
    from statecatcher_amd import train
    calls = []
    real = train.clip_and_adam_step
    monkeypatch.setattr(train, "clip_and_adam_step",
                        lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(4)
    a = torch.nn.Sequential(torch.nn.Linear(32, 48), torch.nn.Linear(48, 8)).to(DEV)
    b = copy.deepcopy(a)
    grads = [torch.randn_like(p) for p in a.parameters()]
    oa = torch.optim.Adam(a.parameters(), lr=1e-2)
    ob = torch.optim.Adam(b.parameters(), lr=1e-2, foreach=False)
    tr = train.SegmentTrainer(a, None, oa, max_grad_norm=max_norm)
    for _ in range(3):
        for p, g in zip(a.parameters(), grads):
            p.grad = g.clone()
        for p, g in zip(b.parameters(), grads):
            p.grad = g.clone()
        tr._clip_and_step()
        torch.nn.utils.clip_grad_norm_(b.parameters(), max_norm)
        ob.step()
    assert len(calls) == 3
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=2e-6, atol=1e-7)


def _image_ref(w, block_d, kp, want_t):
    from statecatcher_amd import ops
    rows, cols = (1, w.shape[0]) if w.dim() == 1 else tuple(w.shape)
    w2 = w.reshape(rows, cols)
    img = ops.step_blocked_rows(w2, block_d, dtype=torch.bfloat16) if block_d \
        else w2.to(torch.bfloat16)
    pad = torch.zeros(rows, kp, dtype=torch.bfloat16, device=w.device)
    pad[:, :cols] = img
    return pad, (img.t().contiguous() if want_t else None)


def test_weight_images_bit_exact_and_cached():
    from statecatcher_amd import ops
    g = torch.Generator(device=DEV).manual_seed(7)
    ws = [torch.randn(3584, 512, device=DEV, generator=g),      # gate weight, step-blocked
          torch.randn(3584, 80, device=DEV, generator=g),       # layer 0, padded to 128
          torch.randn(1024, 512, device=DEV, generator=g),      # output projection
          torch.randn(1024, device=DEV, generator=g),           # its bias
          torch.randn(448, 70, device=DEV, generator=g),        # ragged tiles
          torch.randn(37, 129, device=DEV, generator=g)[:, 1:]]  # strided, unaligned rows
    ws[1][0, 0] = float("nan")
    specs = [(ws[0], 512, 512, True), (ws[1], 512, 128, False), (ws[2], 0, 512, True),
             (ws[3], 0, 1024, False), (ws[4], 64, 70, True), (ws[5], 0, 136, True)]
    imgs = ops.weight_images(specs)
    for (w, bd, kp, wt), (img, img_t) in zip(specs, imgs):
        ref, ref_t = _image_ref(w, bd, kp, wt)
        assert torch.equal(img.reshape(ref.shape).view(torch.int16), ref.view(torch.int16))
        if wt:
            assert torch.equal(img_t.view(torch.int16), ref_t.view(torch.int16))
        else:
            assert img_t is None
    # unchanged weights: cached images; an in-place update (version bump) rebuilds
    again = ops.weight_images(specs)
    assert all(a[0] is b[0] for a, b in zip(imgs, again))
    with torch.no_grad():
        ws[0].mul_(2.0)
    third = ops.weight_images(specs)
    assert third[0][0] is not imgs[0][0] and third[2][0] is imgs[2][0]
    ref, _ = _image_ref(ws[0], 512, 512, False)
    assert torch.equal(third[0][0].view(torch.int16), ref.view(torch.int16))


def test_module_with_weight_images_equals_self_cast(monkeypatch):
    """LucyRNNtriton under bf16 autocast on the cached weight images (one sc_weight_images
    launch) equals the per-layer casts it replaces bit for bit: logits, carried states and every
    parameter gradient (layer 0 padded to the TN kernel's K, step-blocked gate rows, output
    projection W / W^T / b)."""
    from statecatcher_amd import LucyRNNConfig, LucyRNNtriton
    torch.manual_seed(3)
    cfg = LucyRNNConfig(80, 128, 3, 256, kernel_impl="triton", fused_ops=True, layer_norm=False)
    m = LucyRNNtriton(cfg).to(DEV)
    with torch.no_grad():
        m.output_proj.weight.normal_(0, 0.05)
        m.output_proj.bias.normal_(0, 0.05)
    x = torch.randn(2, 192, 80, device=DEV)

    def run():
        m.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            logits, (h, s) = m(x)
        (logits.float().square().mean() + sum(t.sum() for t in h[0])).backward()
        return [logits.float(), *h[0], *s[0]] + [p.grad.clone() for p in m.parameters()]

    with_images = run()
    assert m._weight_images(x.to(DEV))[0] is None   # outside autocast: no images
    monkeypatch.setattr(type(m), "_weight_images", lambda self, x: (None, None, None))
    self_cast = run()
    for a, b in zip(with_images, self_cast):
        assert torch.equal(a, b)
