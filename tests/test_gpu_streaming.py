"""GPU parity of the streaming LucyRNN step + fused greedy decode (statecatcher_amd/streaming.py,
csrc/lucy_step.hip, sc_ctc_greedy_step in csrc/decode.hip) — SURVEY §8(f) row 2.

* the reference's own infer-mode outputs (tests/golden/native.npz, lucyrnn.LucyRNN run with
  is_training=False: fused/unfused, LayerNorm on/off, frame stacking, carried state) replayed
  frame by frame: logits and final (h, s) at fp32 tolerance 1e-4 relative;
* larger random models against the numpy oracle's cell loop (oracle/native.py, lucyrnn.py:44-70)
  with ragged frame masks, every (fused, layer_norm) combination, hipGraph on and off, 1 and 4
  frames per call;
* tokens: bit-exact with oracle/decode.py (decoder.py:3-30) applied to the same logits.
"""
import numpy as np
import pytest
import torch

from oracle import decode as odec
from oracle import native as onat
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def close(got, ref, rtol=1e-4, afrac=1e-5):
    got = got.detach().double().cpu().numpy() if isinstance(got, torch.Tensor) else got
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=afrac * max(np.abs(ref).max(), 1e-30))


def golden_model(z, name):
    import statecatcher_amd as sc
    train, fused, ln, prefix, stack, carry = [int(v) for v in z[name + "/cfg"]]
    cfg = sc.LucyRNNConfig(input_dim=12, hidden_dim=16, num_layers=2, vocab_size=10,
                           kernel_impl="native", is_training=False, fused_ops=bool(fused),
                           layer_norm=bool(ln), stack_order=stack)
    m = sc.LucyRNN(cfg)
    m.load_state_dict({k[len(name) + 7:]: torch.as_tensor(z[k]) for k in z.files
                       if k.startswith(name + "/param/")})
    return m.to(DEV), bool(carry)


@pytest.mark.parametrize("name", ["infer_carry", "infer_ln0", "infer_ln1", "infer_stack2",
                                  "infer_unfused"])
@pytest.mark.parametrize("K,graph", [(1, True), (4, True), (3, False)])
def test_streaming_vs_reference_infer_golden(name, K, graph):
    from statecatcher_amd.streaming import StreamingLucyRNN
    z = load_golden("native")
    m, carry = golden_model(z, name)
    st = StreamingLucyRNN(m, batch=2, frames_per_call=K, graph=graph)
    if carry:
        st.reset(([torch.as_tensor(t) for t in z[name + "/h0"]],
                  [torch.as_tensor(t) for t in z[name + "/s0"]]))
    toks, logits = st.decode(torch.as_tensor(z[name + "/x"]).to(DEV), return_logits=True)
    close(logits, z[name + "/logits"])
    h, s = st.state()
    close(torch.stack(h), z[name + "/h"])
    close(torch.stack(s), z[name + "/s"])
    lg = logits.cpu().numpy()
    assert toks == odec.ctc_greedy(lg, [lg.shape[1]] * 2)


def oracle_params(m):
    return {k: v.detach().double().cpu().numpy() for k, v in m.state_dict().items()}


def oracle_stream(p, x, masks, L, fused, ln):
    """lucyrnn.py:172-186 frame loop with the per-frame mask blend of :66-68."""
    B, T, _ = x.shape
    D = p["layers.0.input_proj.weight"].shape[0]
    h = [np.zeros((B, D)) for _ in range(L)]
    s = [np.zeros((B, D)) for _ in range(L)]
    out = []
    for t in range(T):
        it = x[:, t]
        mk = masks[:, t][:, None].astype(np.float64)
        for l in range(L):
            h[l], s[l] = onat.cell(p, f"layers.{l}.", it, h[l], s[l], fused, ln, mask=mk)
            it = h[l]
        out.append(onat._lin(it, p, "output_proj"))
    return np.stack(out, 1), h, s


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("ln", [True, False])
@pytest.mark.parametrize("D,engine", [(128, "frame"), (128, "library"), (200, "auto")])
def test_streaming_vs_oracle_ragged(fused, ln, D, engine):
    import statecatcher_amd as sc
    from statecatcher_amd.streaming import StreamingLucyRNN
    torch.manual_seed(D + 2 * fused + ln)
    L, F, V, B, T = 3, 40, 50, 5, 23
    m = sc.LucyRNN(sc.LucyRNNConfig(input_dim=F, hidden_dim=D, num_layers=L, vocab_size=V,
                                    is_training=False, fused_ops=fused, layer_norm=ln))
    with torch.no_grad():   # the reference zero-inits output_proj; make the logits informative
        m.output_proj.weight.normal_(0.0, 0.3)
        m.output_proj.bias.normal_(0.0, 0.3)
    m = m.to(DEV)
    x = torch.randn(B, T, F)
    lens = torch.tensor([23, 1, 17, 0, 9])
    masks = torch.arange(T)[None, :] < lens[:, None]
    p = oracle_params(m)
    rl, rh, rs = oracle_stream(p, x.double().numpy(), masks.numpy(), L, fused, ln)
    for K, graph in ((1, True), (4, True), (2, False)):
        st = StreamingLucyRNN(m, batch=B, frames_per_call=K, graph=graph, engine=engine)
        assert st.engine == ("library" if D == 200 else engine)
        toks, logits = st.decode(x.to(DEV), masks.to(DEV), return_logits=True)
        close(logits, rl, rtol=1e-4, afrac=1e-4)
        h, s = st.state()
        close(torch.stack(h), np.stack(rh), rtol=1e-4, afrac=1e-4)
        close(torch.stack(s), np.stack(rs), rtol=1e-4, afrac=1e-4)
        lg = logits.cpu().numpy()
        assert toks == odec.ctc_greedy(lg, lens.numpy())


def test_streaming_bf16_tracks_fp32():
    """bf16 GEMMs/activations (fp32 state) drift from the fp32 stream no more than the
    reference's own frame loop run under bf16 autocast (lucyrnn.py:172-184, as train.py runs
    the model under autocast) drifts from its fp32 run."""
    import statecatcher_amd as sc
    from statecatcher_amd.streaming import StreamingLucyRNN
    torch.manual_seed(3)
    m = sc.LucyRNN(sc.LucyRNNConfig(input_dim=80, hidden_dim=512, num_layers=6, vocab_size=256,
                                    is_training=False)).to(DEV)
    with torch.no_grad():
        m.output_proj.weight.normal_(0.0, 0.05)
    x = torch.randn(8, 40, 80, device=DEV)
    _, l32 = StreamingLucyRNN(m, 8, 8).decode(x, return_logits=True)
    _, l16 = StreamingLucyRNN(m, 8, 8, dtype=torch.bfloat16).decode(x, return_logits=True)
    rel = float((l16.float() - l32).norm() / l32.norm())
    z = [torch.zeros(8, 512, device=DEV) for _ in range(6)]
    st, outs = (list(z), list(z)), []
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for t in range(40):
            lg, st = m.step(x[:, t], st)
            outs.append(lg.float())
    rel_ac = float((torch.stack(outs, 1) - l32).norm() / l32.norm())
    assert rel < 1.5 * rel_ac + 1e-3, (rel, rel_ac)


@pytest.mark.parametrize("B", [64, 77])
@pytest.mark.parametrize("fused", [True, False])
def test_frame_engine_equals_library_engine_at_bench_size(fused, B):
    """The fused frame chain (csrc/lucy_frame.hip) against the library-GEMM engine on the stream
    bench's model (6 x 512, V 1024, layer_norm on), 64 / 77 streams with ragged masks, fp32:
    logits, state and tokens.  (>= 64 streams the gate GEMM runs 32-row workgroups; 77 leaves a
    ragged last row tile.)"""
    import statecatcher_amd as sc
    from statecatcher_amd.streaming import StreamingLucyRNN
    torch.manual_seed(7 + fused)
    m = sc.LucyRNN(sc.LucyRNNConfig(input_dim=80, hidden_dim=512, num_layers=6, vocab_size=1024,
                                    is_training=False, fused_ops=fused)).to(DEV)
    with torch.no_grad():
        m.output_proj.weight.normal_(0.0, 0.05)
    T = 24
    x = torch.randn(B, T, 80, device=DEV)
    lens = torch.randint(0, T + 1, (B,))
    masks = (torch.arange(T)[None, :] < lens[:, None]).to(DEV)
    out = {}
    for engine in ("frame", "library"):
        st = StreamingLucyRNN(m, B, 8, engine=engine)
        toks, lg = st.decode(x, masks, return_logits=True)
        out[engine] = (toks, lg.float(), st.state())
    (tf, lf, (hf, sf)), (tl, ll, (hl, sl)) = out["frame"], out["library"]
    rel = float((lf - ll).norm() / ll.norm())
    print(f"frame vs library engine (fused={fused}): logits rel {rel:.2e}")
    assert rel < 1e-4
    for a, b in zip(hf + sf, hl + sl):
        assert float((a - b).norm() / max(float(b.norm()), 1e-30)) < 1e-4
    lg = ll.cpu().numpy()
    assert tf == odec.ctc_greedy(lf.cpu().numpy(), lens.numpy())


@pytest.mark.parametrize("K", [8, 2])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("fused", [True, False])
def test_wavefront_schedule_equals_frame_by_frame_schedule(fused, dtype, K):
    """The block as stages over (frame, layer) (schedule="wavefront": multi-job launches of
    sc_lucy_frame_gemm_multi / _cellb_multi, one output projection over the block, one greedy
    launch) against the frame-by-frame chain (schedule="frame") on the stream bench's model
    (6 x 512, V 1024, layer_norm on), 77 ragged streams, blocks of 8 and of 2 (< L) frames:
    tokens, logits and state BITWISE equal (same kernels, same arithmetic per (frame, layer))."""
    import statecatcher_amd as sc
    from statecatcher_amd.streaming import StreamingLucyRNN
    torch.manual_seed(21 + fused)
    m = sc.LucyRNN(sc.LucyRNNConfig(input_dim=80, hidden_dim=512, num_layers=6, vocab_size=1024,
                                    is_training=False, fused_ops=fused)).to(DEV)
    with torch.no_grad():
        m.output_proj.weight.normal_(0.0, 0.05)
    B, T = 77, 20
    x = torch.randn(B, T, 80, device=DEV)
    lens = torch.randint(0, T + 1, (B,))
    masks = (torch.arange(T)[None, :] < lens[:, None]).to(DEV)
    out = {}
    for sched in ("wavefront", "frame"):
        st = StreamingLucyRNN(m, B, K, dtype=dtype, schedule=sched)
        assert st.engine == "frame" and st.schedule == sched
        toks, lg = st.decode(x, masks, return_logits=True)
        out[sched] = (toks, lg, st.state())
    (tw, lw, (hw, sw)), (tf, lf, (hf, sf)) = out["wavefront"], out["frame"]
    assert tw == tf
    assert torch.equal(lw, lf)
    for a, b in zip(hw + sw, hf + sf):
        assert torch.equal(a, b)


def test_streaming_reset_subset_and_blocks_equal_one_pass():
    """Feeding an utterance in two calls equals one call; resetting one stream restarts only
    that stream (its tokens equal a fresh decoder's)."""
    import statecatcher_amd as sc
    from statecatcher_amd.streaming import StreamingLucyRNN
    torch.manual_seed(5)
    m = sc.LucyRNN(sc.LucyRNNConfig(input_dim=20, hidden_dim=64, num_layers=2, vocab_size=12,
                                    is_training=False, fused_ops=True))
    with torch.no_grad():
        m.output_proj.weight.normal_(0.0, 0.5)
    m = m.to(DEV)
    x = torch.randn(3, 16, 20, device=DEV)
    one = StreamingLucyRNN(m, 3, 4)
    e_all = torch.cat([one.step(x[:, i:i + 4]).clone() for i in range(0, 16, 4)], 1)
    two = StreamingLucyRNN(m, 3, 4)
    for i in range(0, 8, 4):
        two.step(x[:, i:i + 4])
    two.reset(streams=[1])
    e_tail = torch.cat([two.step(x[:, i:i + 4]).clone() for i in range(8, 16, 4)], 1)
    fresh = StreamingLucyRNN(m, 3, 4)
    e_fresh = torch.cat([fresh.step(x[:, i:i + 4]).clone() for i in range(8, 16, 4)], 1)
    assert torch.equal(e_tail[[0, 2]], e_all[[0, 2], 8:])
    assert torch.equal(e_tail[1], e_fresh[1])


@pytest.mark.parametrize("fused", [True, False])
def test_frame_engine_odd_blocks_reset_and_state_equal_frame_by_frame(fused):
    """3 frames per captured call equal 1-frame eager calls bitwise, through a reset with given
    state after an odd frame count and a ragged mask; state() after the last call too."""
    import statecatcher_amd as sc
    from statecatcher_amd.streaming import StreamingLucyRNN
    torch.manual_seed(11 + fused)
    m = sc.LucyRNN(sc.LucyRNNConfig(input_dim=24, hidden_dim=64, num_layers=3, vocab_size=40,
                                    is_training=False, fused_ops=fused))
    with torch.no_grad():
        m.output_proj.weight.normal_(0.0, 0.4)
    m = m.to(DEV)
    B, T = 4, 15
    x = torch.randn(B, T, 24, device=DEV)
    mask = (torch.rand(B, T, device=DEV) > 0.2).float()
    h0 = [torch.randn(B, 64, device=DEV) * 0.3 for _ in range(3)]
    s0 = [torch.randn(B, 64, device=DEV) * 0.3 for _ in range(3)]
    ref = StreamingLucyRNN(m, B, 1, graph=False)
    blk = StreamingLucyRNN(m, B, 3, graph=True)
    assert ref.engine == blk.engine == "frame" and blk.graph is not None
    e_ref, l_ref = [], []
    for t in range(T):
        if t == 3:
            ref.reset(hidden_states=(h0, s0))
        e_ref.append(ref.step(x[:, t:t + 1], mask[:, t:t + 1]).clone())
        l_ref.append(ref.logits[0].clone())
    e_blk, l_blk = [], []
    for c in range(T // 3):
        if c == 1:
            blk.reset(hidden_states=(h0, s0))
        e_blk.append(blk.step(x[:, 3 * c:3 * c + 3], mask[:, 3 * c:3 * c + 3]).clone())
        l_blk.append(blk.logits.clone())
    assert torch.equal(torch.cat(e_ref, 1), torch.cat(e_blk, 1))
    assert torch.equal(torch.stack(l_ref), torch.cat(l_blk))
    (hr, sr), (hb, sb) = ref.state(), blk.state()
    for a, b in zip(hr + sr, hb + sb):
        assert torch.equal(a, b)


def test_greedy_frames_kernel_equals_greedy_steps():
    """sc_ctc_greedy_frames over F frames == F sc_ctc_greedy_step calls (ties, NaN, masks)."""
    from statecatcher_amd import ops
    g = torch.Generator().manual_seed(3)
    F, B, V = 9, 37, 50
    lg = torch.randint(0, 6, (F, B, V), generator=g).float().to(DEV)   # many ties
    lg[2, 5, 7] = float("nan")
    mask = (torch.rand(F, B, generator=g) > 0.3).float().to(DEV)
    for dt in (torch.float32, torch.bfloat16):
        x = lg.to(dt)
        p1 = torch.full((B,), -1, dtype=torch.int32, device=DEV)
        p2 = p1.clone()
        e1 = torch.empty(F, B, dtype=torch.int32, device=DEV)
        e2 = torch.empty(F, B, dtype=torch.int32, device=DEV)
        for f in range(F):
            ops.ctc_greedy_step(x[f], p1, e1[f], mask=mask[f], blank=0)
        ops.ctc_greedy_frames(x, p2, e2, mask=mask, blank=0)
        assert torch.equal(e1, e2) and torch.equal(p1, p2)


def test_greedy_step_kernel_ties_nan_masks_vs_oracle():
    """sc_ctc_greedy_step frame by frame == decoder.py over the sequence (ties -> lowest index,
    NaN wins, masked frames past the length emit nothing), bf16 and fp32 logits."""
    from statecatcher_amd import ops
    rng = np.random.default_rng(7)
    B, T, V = 6, 40, 37
    for dt in (torch.float32, torch.bfloat16):
        x = rng.integers(0, 4, (B, T, V)).astype(np.float32)    # many ties
        x[1, 5, 3] = np.nan
        x[2, :, :] = 0.0                                         # all-tie rows -> blank (0)
        lens = np.array([40, 33, 40, 0, 1, 12])
        xt = torch.as_tensor(x).to(dt)
        ref = odec.ctc_greedy(xt.float().numpy(), lens)
        prev = torch.full((B,), -1, dtype=torch.int32, device=DEV)
        emit = torch.empty(T, B, dtype=torch.int32, device=DEV)
        xd = xt.to(DEV)
        for t in range(T):
            mk = torch.as_tensor((t < lens).astype(np.float32), device=DEV)
            ops.ctc_greedy_step(xd[:, t], prev, emit[t], mask=mk)
        got = [[int(v) for v in row if v >= 0] for row in emit.t().cpu()]
        assert got == ref
