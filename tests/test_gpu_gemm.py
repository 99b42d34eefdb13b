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
                                   (1024, 768, 768)])
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


def test_wgrad_mfma_structured_exact():
    """Integer-valued operands: every partial sum is exact in fp32, so the result must be bitwise
    equal — pins the fragment maps (i, j, L order) independent of rounding."""
    L, I, J = 2048, 512, 256
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
