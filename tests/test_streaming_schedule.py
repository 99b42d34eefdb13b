"""CPU check of the streaming wavefront schedule (StreamingLucyRNN._block_wavefront): the launches
it issues, replayed symbolically, respect every data dependency of the frame-by-frame chain and
never overwrite a buffer before its reader has run.

The kernels are replaced by recorders; each job's input / output buffers are identified by their
data pointers.  Replaying the recorded launch sequence in order, every (layer, frame) must
  * read its layer input (x[j] for layer 0, xo[l-1] otherwise) holding frame j's value of the
    previous layer, i.e. written by (l - 1, j) and not yet overwritten by (l - 1, j + 1);
  * update its state h[l], s[l] after (l, j - 1) did;
  * run its four kernels in order, each after the previous one's launch;
and the output projection / greedy launch must come after every frame's last layer.  The GPU
tests (tests/test_gpu_streaming.py) check the same schedule bitwise against the frame-by-frame
chain; this one runs without a GPU, for any (K, L)."""
import types

import pytest
import torch


def _fake_stream(L, K, B=3, D=32, Din=16, V=10, fused=False, ln=True):
    from statecatcher_amd.streaming import StreamingLucyRNN
    z = lambda *s: torch.zeros(*s)   # noqa: E731
    st = StreamingLucyRNN.__new__(StreamingLucyRNN)
    st.cfg = types.SimpleNamespace(fused_ops=fused)
    st.L, st.K, st.B, st.D, st.V, st.blank = L, K, B, D, V, 0
    st.x, st.mask = z(K, B, Din), torch.ones(K, B)
    ng = 5 if fused else 4
    lnp = (z(D), z(D)) if ln else None
    st.layers = [dict(w_in=z(D, Din if l == 0 else D), b_in=z(D), ln_in=lnp, lnz=lnp, lnh=lnp,
                      w_g=z(ng * D, D), b_g=z(ng * D), w_h=z(D, D), b_h=z(D)) for l in range(L)]
    st.wf = [dict(fa=z(B, D), fz=z(B, D), fy=z(B, D), fhp=z(B, D), st_a=z((D + 31) // 32, B, 4),
                  st_z=z(D // 16, B, 4), st_h=z(D // 16, B, 4)) for _ in range(L)]
    st.xo = [z(B, D) for _ in range(L)]
    st.h = [z(B, D) for _ in range(L)]
    st.s = [z(B, D) for _ in range(L)]
    st.xlast = z(K, B, D)
    st.w_out, st.b_out = z(V, D), z(V)
    st.logits = z(K, B, V)
    st.prev = torch.full((B,), -1, dtype=torch.int32)
    st.emit = torch.full((K, B), -1, dtype=torch.int32)
    return st


@pytest.mark.parametrize("L,K", [(6, 8), (6, 2), (3, 1), (2, 5), (10, 3)])
@pytest.mark.parametrize("fused", [False, True])
def test_wavefront_schedule_respects_dependencies(monkeypatch, L, K, fused):
    from statecatcher_amd import ops
    st = _fake_stream(L, K, fused=fused)
    launches = []   # (kind, [(in_ptr, out_ptr, h_ptr)])
    monkeypatch.setattr(ops._lib, "stream_of", lambda t: None)
    monkeypatch.setattr(ops, "lucy_frame_gemm_multi",
                        lambda epi, wdt, jobs, stream, eps=1e-5: launches.append(
                            (("gemm", epi), [(j.x, j.y, j.s) for j in jobs])))
    monkeypatch.setattr(ops, "lucy_frame_cellb_multi",
                        lambda jobs, stream, eps=1e-5: launches.append(
                            ("cellb", [(j.z, j.out, j.h) for j in jobs])))
    monkeypatch.setattr(ops, "lucy_frame_gemm",
                        lambda epi, x, w, bias, y, **kw: launches.append(
                            ("out", [(x.data_ptr(), y.data_ptr(), None)])))
    monkeypatch.setattr(ops, "ctc_greedy_frames",
                        lambda logits, prev, emit, mask=None, blank=0: launches.append(("greedy", [])))
    st._block_wavefront()

    ptr = lambda t: t.data_ptr()   # noqa: E731
    # the value each buffer holds during the replay: (layer, frame) of its producer
    holds = {ptr(st.x[j]): ("input", j) for j in range(K)}
    n_kernels = 3 if fused else 4
    step_done = {}   # (l, j) -> launch index of its cellb
    for li, (kind, jobs) in enumerate(launches):
        if kind in ("out", "greedy"):
            continue
        for (inp, out, hst) in jobs:
            if kind == "cellb":
                l = [i for i in range(L) if ptr(st.h[i]) == hst][0]
                j = [jj for jj in range(K) if (l, jj) not in step_done][0]
                # its layer's state after its previous frame, its GEMMs before it
                assert j == 0 or step_done[(l, j - 1)] < li
                step_done[(l, j)] = li
                exp_out = ptr(st.xlast[j]) if l == L - 1 else ptr(st.xo[l])
                assert out == exp_out
                holds[out] = (l, j)
            elif any(inp == ptr(st.x[j]) for j in range(K)) or any(inp == ptr(t) for t in st.xo):
                # an input projection (the only GEMM reading x or xo): its input must hold the
                # previous layer's value of the frame this layer is at
                if any(out == ptr(w["fa"]) for w in st.wf):
                    l = [i for i in range(L) if ptr(st.wf[i]["fa"]) == out][0]
                    j = len([1 for (ll, _jj) in step_done if ll == l])
                    want = ("input", j) if l == 0 else (l - 1, j)
                    assert holds[inp] == want, (li, l, j, holds[inp], want)
    # every (layer, frame) ran, each layer's frames in order
    assert sorted(step_done) == sorted((l, j) for l in range(L) for j in range(K))
    # one output projection and one greedy launch, after every frame's last layer
    kinds = [k for k, _ in launches]
    assert kinds.count("out") == 1 and kinds.count("greedy") == 1
    last_cell = max(step_done.values())
    assert kinds.index("out") > last_cell and kinds.index("greedy") > kinds.index("out")
    # launch count: (3 or 4 kernels) per stage, K + L - 1 stages (with <= 8 jobs per launch)
    stages = K + L - 1
    per_stage = [min(L, K, t + 1, K + L - 1 - t) for t in range(stages)]
    want = sum(n_kernels * ((n + 7) // 8) for n in per_stage) + 2
    assert len(launches) == want, (len(launches), want)
