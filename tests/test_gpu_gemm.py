"""GPU parity of the MFMA split-L weight-gradient GEMM (gemm.hip, sc_gemm_wgrad_bf16 + the
sc_colsum slab sum) against an fp32 torch reference of the same op, dW = dy^T x.

Tolerance: bf16 inputs are exact in fp32, products are exact in the fp32 MFMA accumulator, so
the only error is fp32 summation order over L: 1e-5 of the largest |dW| (observed ~1e-6)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def ops():
    from statecatcher_amd import ops as o
    return o


def _ref(dy, x):
    return dy.float().t() @ x.float()


@pytest.mark.parametrize("L,I,J", [(48000, 3584, 512),   # gate projection, C2 (224-row tiles)
                                   (48000, 1024, 512),   # output projection
                                   (6400, 3584, 512),
                                   (4096, 512, 256),
                                   (1024, 768, 768),
                                   (14336, 768, 768),    # C4 out_proj: 9 tiles x 28 splits
                                   (4096, 4096, 768),    # C4 FFN up: 48 x 5, uneven ranges
                                   (6400, 768, 2048),    # C4 FFN down: 24 x 10
                                   # 128-column tiles (round 6): layer 0's 80 features padded
                                   (48000, 3584, 128),   # to 128 (224-row tiles, 16 splits)
                                   (4096, 512, 384),     # 256-row tiles, 3 column tiles
                                   (1024, 1024, 128)])
def test_wgrad_mfma_vs_fp32(L, I, J):
    from statecatcher_amd import _lib
    assert _lib.load().sc_gemm_wgrad_splits(L, I, J) > 0
    g = torch.Generator(device=DEV).manual_seed(L + I + J)
    # asymmetric, non-trivial operands (catches row/column swaps and fragment-order bugs)
    dy = torch.randn(L, I, device=DEV, generator=g).to(torch.bfloat16)
    x = (torch.randn(L, J, device=DEV, generator=g) +
         torch.arange(J, device=DEV) / J).to(torch.bfloat16)
    dw = ops().wgrad_mfma(dy, x)
    ref = _ref(dy, x)
    err = (dw - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


def test_wgrad_splits_fill_the_chip():
    """The split count fills the 256 CUs for any tile count (not only powers of two), and each
    split keeps at least 8 K-blocks of 64 rows."""
    from statecatcher_amd import _lib
    lib = _lib.load()
    assert lib.sc_gemm_wgrad_splits(48000, 3584, 512) == 8     # C2 gates: 32 tiles (224 rows)
    assert lib.sc_gemm_wgrad_splits(48000, 1024, 512) == 32    # C2 output projection: 8 tiles
    assert lib.sc_gemm_wgrad_splits(48000, 768, 768) == 28     # 9 tiles
    assert lib.sc_gemm_wgrad_splits(48000, 4096, 768) == 5     # 48 tiles
    assert lib.sc_gemm_wgrad_splits(48000, 768, 2048) == 10    # 24 tiles
    assert lib.sc_gemm_wgrad_splits(1024, 768, 768) == 2       # 16 K-blocks: 8 per split
    assert lib.sc_gemm_wgrad_splits(512, 4096, 4096) == 1
    assert lib.sc_gemm_wgrad_splits(48000, 3584, 128) == 16   # layer 0: 16 tiles of 224 x 128
    assert lib.sc_gemm_wgrad_splits(48000, 3584, 80) == 0     # (the caller pads to 128)


@pytest.mark.parametrize("J", [256, 128])
def test_wgrad_mfma_structured_exact(J):
    """Integer-valued operands: every partial sum is exact in fp32, so the result must be bitwise
    equal — pins the fragment maps (i, j, L order) independent of rounding, for the 256- and the
    128-column tile."""
    L, I = 2048, 512
    li = torch.arange(L, device=DEV)
    dy = ((li[:, None] * 3 + torch.arange(I, device=DEV)[None, :] * 7) % 5 - 2).to(torch.bfloat16)
    x = ((li[:, None] * 5 + torch.arange(J, device=DEV)[None, :] * 11) % 7 - 3).to(torch.bfloat16)
    dw = ops().wgrad_mfma(dy, x)
    assert torch.equal(dw, _ref(dy, x))


def test_wgrad_mfma_step_blocked_unpermute():
    """blocked_d: dy's columns in step-blocked order (column block, gate, unit); the slab sum
    writes dW rows back in the reference (gate, unit) order."""
    L, D, J = 4096, 512, 512
    g = torch.Generator(device=DEV).manual_seed(3)
    dy_ref = torch.randn(L, 7 * D, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(L, J, device=DEV, generator=g).to(torch.bfloat16)
    # reference column order (gate, unit) -> blocked (block, gate, unit-in-block)
    dy_blk = dy_ref.view(L, 7, D // 64, 64).permute(0, 2, 1, 3).reshape(L, 7 * D).contiguous()
    dw = ops().wgrad_mfma(dy_blk, x, blocked_d=D)
    ref = _ref(dy_ref, x)
    assert (dw - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()


def test_wgrad_unsupported_shape_falls_back():
    """Shapes outside the tiling return None from wgrad_mfma; wgrad_splitk still answers."""
    dy = torch.randn(1000, 3584, device=DEV).to(torch.bfloat16)   # L % 64 != 0
    x = torch.randn(1000, 80, device=DEV).to(torch.bfloat16)
    assert ops().wgrad_mfma(dy, x) is None
    dw = ops().wgrad_splitk(dy, x)
    ref = _ref(dy, x)
    assert (dw - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()


def test_wgrad_i448_is_rejected_by_the_split_gate():
    """I=448 is a multiple of 224 but not at the 256-workgroup shape: the split gate says 0 and
    the launch itself refuses (the C-ABI contract of statecatcher.h)."""
    from statecatcher_amd import _lib
    lib = _lib.load()
    assert lib.sc_gemm_wgrad_splits(4096, 448, 512) == 0
    dy = torch.randn(4096, 448, device=DEV).to(torch.bfloat16)
    x = torch.randn(4096, 512, device=DEV).to(torch.bfloat16)
    assert ops().wgrad_mfma(dy, x) is None
    part = torch.empty(1, 448, 512, device=DEV)
    rc = lib.sc_gemm_wgrad_bf16(dy.data_ptr(), 448, x.data_ptr(), 512, part.data_ptr(), 4096, 448,
                                512, 1, None)
    assert rc != 0


@pytest.mark.parametrize("N", [7 * 5 * 3, 7 * 2 * 64 + 0])
def test_colsum_perm_with_unaligned_rows(N):
    """sc_colsum's (A, B) un-permutation on a view whose rows are not 16-byte pieces (the padded
    path): the permutation applies to the unpadded width."""
    A, Bf = (5, 7) if N == 105 else (2, 7)
    M = 300
    big = torch.randn(M, N + 3, device=DEV)
    x = big[:, 1:N + 1]   # unaligned base and row pitch
    out = ops().colsum(x, (A, Bf))
    ref = x.double().sum(0).view(A, Bf, -1).transpose(0, 1).reshape(-1)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4)


# ----------------------------------------------------------- frame-major TN GEMM (tn_gemm.hip) --
# C = A B^T in bf16 with fp32 accumulation: products of bf16 values are exact in fp32, so the
# kernel differs from an fp32 reference only by summation order (~1e-6 relative) and then by the
# final bf16 rounding (<= 2^-8 relative); tolerance 2^-8 of the value + 1e-5 of the largest |C|.
def _tn_ref(a, b):
    return a.float() @ b.float().t()


def _tn_check(c, ref):
    assert c.dtype == torch.bfloat16 and c.shape == ref.shape
    err = (c.float() - ref).abs()
    tol = ref.abs() * 2.0 ** -8 + 1e-5 * ref.abs().max()
    assert bool((err <= tol).all()), (err - tol).max().item()


@pytest.mark.parametrize("M,N,K,tm", [(48000, 3584, 512, 0),    # gate forward, layers 1-5 (C2)
                                      (48000, 3584, 128, 0),    # layer 0 (Din 80 padded to 128)
                                      (48000, 512, 3584, 0),    # gate input gradient
                                      (48000, 512, 1024, 0),    # output-projection input gradient
                                      (5000, 1024, 512, 128),   # ragged rows, 128-row tiles
                                      (193, 256, 64, 0),        # one row past a panel
                                      (7, 512, 64, 128),        # fewer rows than a fragment
                                      # the 256 x 256 four-phase kernel
                                      (48000, 3584, 512, 256), (48000, 3584, 128, 256),
                                      (48000, 512, 3584, 256), (48000, 1024, 512, 256),
                                      (5000, 1024, 64, 256),    # one K-tile per output tile
                                      (300, 512, 192, 256),     # odd K-tile count, partial panel
                                      (7, 256, 128, 256),       # fewer rows than a fragment
                                      # the 256 x 256 ping-pong schedule (tile_m 257)
                                      (48000, 3584, 512, 257), (48000, 512, 3584, 257),
                                      (48000, 1024, 512, 257), (5000, 1024, 64, 257),
                                      (300, 512, 192, 257), (7, 256, 128, 257)])
def test_tn_gemm_vs_fp32(M, N, K, tm):
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    a = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    b = (torch.randn(N, K, device=DEV, generator=g) + torch.arange(K, device=DEV) / K).to(torch.bfloat16)
    assert ops().tn_ok(a, b)
    _tn_check(ops().gemm_tn(a, b, tm), _tn_ref(a, b))


@pytest.mark.parametrize("tm", [128, 192, 256, 257])
def test_tn_gemm_structured_exact(tm):
    """Small-integer operands: every sum is exact in fp32 and |C| <= 256 is exact in bf16, so the
    result must equal the reference bitwise — pins the fragment maps, the swizzle and the
    column order of the packed stores independent of rounding."""
    M, N, K = 1000, 512, 192
    mi = torch.arange(M, device=DEV)[:, None]
    a = ((mi * 3 + torch.arange(K, device=DEV)[None, :] * 7) % 5 - 2).to(torch.bfloat16)
    ni = torch.arange(N, device=DEV)[:, None]
    b = (((ni * 5 + torch.arange(K, device=DEV)[None, :] * 11) % 3) - 1).to(torch.bfloat16)
    ref = _tn_ref(a, b)
    assert ref.abs().max() <= 256
    assert torch.equal(ops().gemm_tn(a, b, tm).float(), ref)


def test_tn_gemm_strided_operands_and_row_bound():
    """Leading dimensions wider than K / N, and C rows >= M left untouched (the buffer
    descriptor's range drops the stores of a partial panel)."""
    from statecatcher_amd import _lib
    M, N, K = 300, 512, 128
    g = torch.Generator(device=DEV).manual_seed(5)
    abig = torch.randn(M, K + 40, device=DEV, generator=g).to(torch.bfloat16)
    bbig = torch.randn(N, K + 8, device=DEV, generator=g).to(torch.bfloat16)
    a, b = abig[:, :K], bbig[:, :K]
    cbig = torch.full((M + 100, N + 64), 7.0, device=DEV, dtype=torch.bfloat16)
    rc = _lib.load().sc_gemm_tn_bf16(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0),
                                     cbig.data_ptr(), cbig.stride(0), M, N, K, 0, None)
    assert rc == 0
    torch.cuda.synchronize()
    _tn_check(cbig[:M, :N], _tn_ref(a, b))
    assert bool((cbig[M:] == 7).all()) and bool((cbig[:, N:] == 7).all())


def test_tn_gemm_rejects_bad_shapes():
    from statecatcher_amd import _lib
    lib = _lib.load()
    a = torch.zeros(64, 80, device=DEV, dtype=torch.bfloat16)
    b = torch.zeros(256, 80, device=DEV, dtype=torch.bfloat16)
    c = torch.zeros(64, 256, device=DEV, dtype=torch.bfloat16)
    assert lib.sc_gemm_tn_bf16(a.data_ptr(), 80, b.data_ptr(), 80, c.data_ptr(), 256, 64, 256, 80,
                               0, None) != 0   # K % 32
    assert lib.sc_gemm_tn_bf16(a.data_ptr(), 80, b.data_ptr(), 80, c.data_ptr(), 256, 64, 200, 64,
                               0, None) != 0   # N % 256
    assert not ops().tn_ok(a, b)


def test_autocast_linear_wgrad_split_head():
    """AutocastLinearFn's weight gradient for N not a multiple of 256 (the xLSTM q|k|v|o|i|f
    projection, N = 2312 at C4): the first N - N % 256 rows on the MFMA kernel, the rest on the
    library; against fp32 torch at 1e-5 of the largest |dW| (fp32 summation order)."""
    g = torch.Generator(device=DEV).manual_seed(11)
    x = torch.randn(4096, 768, device=DEV, generator=g).to(torch.bfloat16).float()
    w = torch.randn(2312, 768, device=DEV, generator=g) * 0.02
    dy = torch.randn(4096, 2312, device=DEV, generator=g).to(torch.bfloat16)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops().autocast_linear(xr, wr)
    y.backward(dy)
    ref = dy.float().t() @ x
    err = (wr.grad - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-5, err


def test_autocast_linear_bias_from_sums_only_the_gate_columns():
    """bias_from = 2304 (the xLSTM projection: q|k|v|o bias pieces are constant zeros): the bias
    gradient of columns >= bias_from equals the full column sum, the leading part is 0."""
    g = torch.Generator(device=DEV).manual_seed(12)
    x = torch.randn(4096, 768, device=DEV, generator=g)
    w = torch.randn(2312, 768, device=DEV, generator=g) * 0.02
    b = torch.zeros(2312, device=DEV)
    b[2304:] = torch.randn(8, device=DEV, generator=g)
    dy = torch.randn(4096, 2312, device=DEV, generator=g).to(torch.bfloat16)
    bq = b.clone().requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = ops().autocast_linear(x, w, bq, 2304)
    y.backward(dy)
    ref = dy.float().sum(0)
    assert bool((bq.grad[:2304] == 0).all())
    torch.testing.assert_close(bq.grad[2304:], ref[2304:], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("din", [80, 512])
def test_cell_side_stream_wgrad_bitwise(din, monkeypatch):
    """ops.USE_WGRAD_STREAM (SC_WGRAD_STREAM=1): the cell's weight-gradient kernel on a side
    stream beside the input gradient gives bitwise the same gradients as the one-stream order
    (layer 0's Din = 80 takes the library weight gradient on the main stream either way)."""
    o = ops()
    g = torch.Generator(device="cuda").manual_seed(11)
    B, T, D = 4, 200, 512
    x = torch.randn(B, T, din, device="cuda", generator=g)
    w = torch.randn(7 * D, din, device="cuda", generator=g) * 0.05
    b = torch.randn(7 * D, device="cuda", generator=g) * 0.1
    h0 = torch.zeros(B, D, device="cuda")
    s0 = torch.zeros(B, D, device="cuda")
    dout = torch.randn(B, T, D, device="cuda", generator=g).to(torch.bfloat16)

    def run(side):
        monkeypatch.setattr(o, "USE_WGRAD_STREAM", side)
        leaves = [t.clone().requires_grad_(True) for t in (x, w, b)]
        out, s_last, h_last = o.lucy_cell(leaves[0], leaves[1], leaves[2], h0, s0,
                                          cdt=torch.bfloat16)
        out.backward(dout)
        torch.cuda.synchronize()
        return [t.grad for t in leaves]

    for a, c in zip(run(True), run(False)):
        assert torch.equal(a, c)


def test_layer0_cell_weight_gradient_on_the_128_column_tile(monkeypatch):
    """Layer 0 (Din = 80), SC_WGRAD128=1: LucyCellFn's weight gradient on the MFMA kernel's 128-column tile
    over the zero-padded bf16 copy of x and keeps dW's first 80 columns (round 6; the library's
    MT80x256 kernel ran at 12% MFMA).  Against fp32 torch on the dgates and x the kernel received:
    1e-5 of the largest |dW| (fp32 summation order).  The library path it replaces (wgrad_mfma
    forced off) rounds its split-K partials to bf16 and lands ~2.6e-3 away (measured); the bias
    gradient is bitwise the same either way (it does not touch the weight gradient)."""
    o = ops()
    monkeypatch.setattr(o, "USE_WGRAD128", True)   # (opt-in: SC_WGRAD128=1)
    g = torch.Generator(device="cuda").manual_seed(5)
    B, T, D, din = 2, 1600, 512, 80   # B T = 3200 rows, a multiple of 64
    x = torch.randn(B, T, din, device="cuda", generator=g)
    w = torch.randn(7 * D, din, device="cuda", generator=g) * 0.05
    b = torch.randn(7 * D, device="cuda", generator=g) * 0.1
    h0 = torch.zeros(B, D, device="cuda")
    s0 = torch.zeros(B, D, device="cuda")
    dout = torch.randn(B, T, D, device="cuda", generator=g).to(torch.bfloat16)
    seen = []
    orig = o.wgrad_mfma

    def run(mfma):
        def wg(dy, xx, blocked_d=0):
            seen.append((dy.detach().clone(), xx.detach().clone(), blocked_d))
            return orig(dy, xx, blocked_d) if mfma else None
        monkeypatch.setattr(o, "wgrad_mfma", wg)
        leaves = [t.clone().requires_grad_(True) for t in (w, b)]
        out, _, _ = o.lucy_cell(x, leaves[0], leaves[1], h0, s0, cdt=torch.bfloat16)
        out.backward(dout)
        torch.cuda.synchronize()
        return [t.grad for t in leaves]
    gm, gl = run(True), run(False)
    dy, xx, bd = seen[0]
    assert tuple(xx.shape) == (B * T, 128) and bool((xx[:, din:] == 0).all())   # padded copy
    ref = _ref(dy, xx)
    if bd:   # dy's columns step-blocked: the reference order of dW's rows
        ref = ops().step_blocked_rows(ref, bd, inverse=True)
    ref = ref[:, :din]
    assert gm[0].shape == (7 * D, din) and gm[0].is_contiguous()
    err = (gm[0] - ref).abs().max().item() / ref.abs().max().item()
    err_lib = (gl[0] - ref).abs().max().item() / ref.abs().max().item()
    print(f"layer-0 dW vs fp32: MFMA 128-column tile {err:.2e}, library path {err_lib:.2e}")
    assert err <= 1e-5, err
    assert torch.equal(gm[1], gl[1])
