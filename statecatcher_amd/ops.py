"""Autograd wrappers over the HIP C ABI (include/statecatcher.h).

Each op checks device/dtype/shape, allocates outputs through the PyTorch caching allocator,
launches on the current stream and never synchronises the host.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import check, dtype_code, ptr, require_device, stream_of

# Optional per-launch timing (bench.py roofline): when a list, every scan launch appends
# (name, start_event, end_event, algorithmic_bytes) recorded on the launch stream.
LAUNCH_EVENTS = None


class _timed:
    """HIP events around a launch on t's stream (bench.py's per-kernel timing): algorithmic
    bytes (HBM-bound kernels) or flops (MFMA-bound ones) per launch ride along."""

    def __init__(self, name, t, nbytes, flops=0):
        self.rec = LAUNCH_EVENTS is not None
        if self.rec:
            self.name, self.nbytes, self.flops = name, nbytes, flops
            self.stream = torch.cuda.current_stream(t.device)
            self.e0 = torch.cuda.Event(enable_timing=True)
            self.e1 = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        if self.rec:
            self.e0.record(self.stream)
        return self

    def __exit__(self, *exc):
        if self.rec:
            self.e1.record(self.stream)
            LAUNCH_EVENTS.append((self.name, self.e0, self.e1, self.nbytes, self.flops))
        return False


# ----------------------------------------------------------------------------- LucyRNN scan --
def gate_layout(gates):
    """(B, T, D, strides (bt, td, cd, cb)) of a gate tensor in either accepted layout:
    [B,T,7,D] (the reference's) or step-blocked [B,T,D/64,7,64] (include/statecatcher.h)."""
    if gates.dim() == 4 and gates.shape[2] == 7 and gates.stride(3) == 1:
        B, T, _, D = gates.shape
        return B, T, D, (gates.stride(0), gates.stride(1), gates.stride(2), 64)
    if gates.dim() == 5 and gates.shape[3] == 7 and gates.shape[4] == 64 and gates.stride(4) == 1:
        B, T, NB = gates.shape[:3]
        return B, T, NB * 64, (gates.stride(0), gates.stride(1), gates.stride(3), gates.stride(2))
    raise ValueError(f"gates must be [B,T,7,D] or [B,T,D/64,7,64] with unit inner stride, got "
                     f"shape {tuple(gates.shape)} strides {gates.stride()}")


def _scan_fwd(gates, h0, s0, need_ckpt, bias=None, want_h=False, split=False, ln=None):
    """split (16-bit gates): out is the first D columns of a [B,T,3D] buffer whose other two
    blocks are out again and h - out (sc_lucy_scan_fwd_split), returned as the last element.
    ln = (ln_r, rec_in, stat, rec_out, eps): the folded LayerNorm (sc_lucy_scan_fwd_ln; ln_r /
    rec_in None: records out only)."""
    require_device(gates, h0, s0)
    if gates.dim() == 4 and gates.shape[2] == 7 and gates.stride(3) != 1:
        gates = gates.contiguous()
    B, T, D, gs = gate_layout(gates)
    if tuple(h0.shape) != (B, D) or tuple(s0.shape) != (B, D):
        raise ValueError(f"h0/s0 must be [B,D]=({B},{D}); got {tuple(h0.shape)}, {tuple(s0.shape)}")
    # the reference reads h0/s0 as contiguous even when handed a strided view
    h0c = h0.detach().to(torch.float32).contiguous()
    s0c = s0.detach().to(torch.float32).contiguous()
    split = split and gates.dtype in (torch.bfloat16, torch.float16)
    wide = torch.empty(B, T, 3 * D, dtype=gates.dtype, device=gates.device) if split else None
    out = wide[..., :D] if split else torch.empty(B, T, D, dtype=gates.dtype, device=gates.device)
    s_out = torch.empty(B, D, dtype=torch.float32, device=gates.device)
    h_out = torch.empty(B, D, dtype=torch.float32, device=gates.device) if want_h else None
    lib = _lib.load()
    ckpt = None
    if need_ckpt:
        ckpt = torch.empty(lib.sc_lucy_scan_ckpt_numel(B, T, D), dtype=torch.float32,
                           device=gates.device)
    e = gates.element_size()
    nbytes = B * T * D * 8 * e + (ckpt.numel() * 4 if ckpt is not None else 0) + 4 * B * D * 4
    with _timed("lucy_scan_fwd", gates, nbytes):
        if ln is not None:
            ln_r, rec_in, stat, rec_out, eps = ln
            rc = lib.sc_lucy_scan_fwd_ln(ptr(gates), dtype_code(gates), ptr(bias), ptr(h0c), ptr(s0c),
                                         ptr(out), ptr(wide[..., D:2 * D]) if split else None,
                                         ptr(wide[..., 2 * D:]) if split else None, ptr(s_out),
                                         ptr(h_out), B, T, D, *gs, out.stride(0), out.stride(1),
                                         ptr(ckpt), ptr(ln_r), ptr(rec_in), ptr(stat), ptr(rec_out),
                                         float(eps), stream_of(gates))
        elif split:
            rc = lib.sc_lucy_scan_fwd_split(ptr(gates), dtype_code(gates), ptr(bias), ptr(h0c),
                                            ptr(s0c), ptr(out), ptr(wide[..., D:2 * D]),
                                            ptr(wide[..., 2 * D:]), ptr(s_out), ptr(h_out), B, T, D,
                                            *gs, out.stride(0), out.stride(1), ptr(ckpt),
                                            stream_of(gates))
        else:
            rc = lib.sc_lucy_scan_fwd(ptr(gates), dtype_code(gates), ptr(bias), ptr(h0c), ptr(s0c),
                                      ptr(out), ptr(s_out), ptr(h_out), B, T, D, *gs, out.stride(0),
                                      out.stride(1), ptr(ckpt), stream_of(gates))
    check(rc, "sc_lucy_scan_fwd")
    res = (gates, out, s_out, ckpt, h_out) if want_h else (gates, out, s_out, ckpt)
    return res + (wide,) if split else res


def _scan_bwd(gates, ckpt, dout, ds_last, want_dbias, bias=None, ln=None):
    """dgates come back in the layout of `gates` (contiguous).  ln = (ln_r, stat): the folded
    LayerNorm's backward scan (sc_lucy_scan_bwd_ln: dgates = rstd dL/dgate)."""
    B, T, D, gs = gate_layout(gates)
    if dout is None:
        dout = torch.zeros(B, T, D, dtype=gates.dtype, device=gates.device)
    dout = dout.to(gates.dtype)
    if dout.stride(2) != 1:
        dout = dout.contiguous()
    if ds_last is not None:
        ds_last = ds_last.to(torch.float32).contiguous()
    dgates = torch.empty(gates.shape, dtype=gates.dtype, device=gates.device)
    _, _, _, dgs = gate_layout(dgates)
    dh0 = torch.empty(B, D, dtype=torch.float32, device=gates.device)
    ds0 = torch.empty(B, D, dtype=torch.float32, device=gates.device)
    dbias = torch.empty(B, 7, D, dtype=torch.float32, device=gates.device) if want_dbias else None
    e = gates.element_size()
    nbytes = B * T * D * 15 * e + ckpt.numel() * 4 + 3 * B * D * 4
    with _timed("lucy_scan_bwd", gates, nbytes):
        if ln is not None:
            rc = _lib.load().sc_lucy_scan_bwd_ln(
                ptr(gates), dtype_code(gates), ptr(bias), ptr(ckpt), ptr(dout), ptr(ds_last),
                ptr(dgates), ptr(dh0), ptr(ds0), ptr(dbias), B, T, D, *gs, dout.stride(0),
                dout.stride(1), *dgs, ptr(ln[0]), ptr(ln[1]), stream_of(gates))
        else:
            rc = _lib.load().sc_lucy_scan_bwd(
                ptr(gates), dtype_code(gates), ptr(bias), ptr(ckpt), ptr(dout), ptr(ds_last),
                ptr(dgates), ptr(dh0), ptr(ds0), ptr(dbias), B, T, D, *gs, dout.stride(0),
                dout.stride(1), *dgs, stream_of(gates))
    check(rc, "sc_lucy_scan_bwd")
    return dgates, dh0, ds0, dbias


class LucyScanFn(torch.autograd.Function):
    """out, s_last = scan(gates [B,T,7,D], h0 [B,D], s0 [B,D]).

    Forward = lucyrnn_triton.py:179-244 (rnn_forward_unfused_rmsnorm).  Unlike the reference
     the outputs carry gradients to gates, h0 and s0.  out has the gates' dtype;
    s_last is fp32 (state arithmetic is fp32 for every gate dtype).
    """

    @staticmethod
    def forward(ctx, gates, h0, s0):
        need = any(ctx.needs_input_grad)
        gates, out, s_out, ckpt = _scan_fwd(gates, h0, s0, need)
        if need:
            ctx.save_for_backward(gates, ckpt)
            ctx.state_dtypes = (h0.dtype, s0.dtype)
        return out, s_out

    @staticmethod
    def backward(ctx, dout, ds_last):
        gates, ckpt = ctx.saved_tensors
        dgates, dh0, ds0, _ = _scan_bwd(gates, ckpt, dout, ds_last, False)
        hd, sd = ctx.state_dtypes
        return dgates, dh0.to(hd), ds0.to(sd)


def lucy_scan(gates, h0, s0):
    return LucyScanFn.apply(gates, h0, s0)


def colsum(x2d, perm=(1, 1)):
    """fp32 column sums of a row-major [M, N] matrix (sc_colsum, deterministic); perm = (A, B)
    writes input column (a, b, c) of an (A, B, N/(A*B)) factorisation at (b, a, c).  CPU tensors
    (gloo tests of the training loop) use torch.sum — there is no GPU fallback."""
    M, N = x2d.shape
    if x2d.device.type == "cpu":
        out = x2d.sum(0, dtype=torch.float32)
        A, Bf = perm
        return out if A == 1 else out.view(A, Bf, -1).transpose(0, 1).reshape(-1)
    per16 = 16 // x2d.element_size()
    if x2d.stride(1) != 1 or (x2d.data_ptr() % 16) or x2d.stride(0) % per16:
        if N % per16 or perm != (1, 1):
            # rows padded to 16 bytes (the kernel's vector loads); zero columns add nothing.  The
            # (A, B, N/(A*B)) un-permutation is defined on the unpadded width: applied here
            # after the slice, never to the padded columns
            xp = torch.zeros(M, N + (-N) % per16, dtype=x2d.dtype, device=x2d.device)
            xp[:, :N] = x2d
            out = colsum(xp)[:N]
            A, Bf = perm
            return out if A == 1 else out.view(A, Bf, -1).transpose(0, 1).reshape(-1)
        x2d = x2d.contiguous()
    lib = _lib.load()
    out = torch.empty(N, dtype=torch.float32, device=x2d.device)
    wsb = lib.sc_colsum_workspace_bytes(M, N)
    ws = torch.empty(wsb, dtype=torch.uint8, device=x2d.device)
    rc = lib.sc_colsum(ptr(x2d), dtype_code(x2d), M, N, x2d.stride(0), int(perm[0]), int(perm[1]),
                       ptr(out), ptr(ws), wsb, stream_of(x2d))
    check(rc, "sc_colsum")
    return out


def wgrad_splitk(dy, x, blocked_d=0):
    """dW = dy^T x (fp32) for dy [M,N], x [M,K] with M = B*T large: at the training shape
    dW is 3584 x 512 while M = 48000, so a plain GEMM has 28 output tiles for 256 CUs; split M
    into S batched GEMMs and sum the partials in fp32.  blocked_d = D: dy's columns are in
    step-blocked order (step_blocked_rows); the sum writes dW back in the reference's order."""
    M, N = dy.shape
    K = x.shape[1]
    if dy.device.type != "cpu" and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16:
        dw = wgrad_mfma(dy, x, blocked_d)
        if dw is not None:
            return dw
    S = 1
    # measured on MI355X at M=48000, N=3584, K=512 (tools/gemm_probe.py): S=1 410 TF/s,
    # S=8 760, S=16 860
    while S < 16 and M % (2 * S) == 0 and M // (2 * S) >= 2048 and \
            ((N + 255) // 256) * ((K + 255) // 256) * S < 512:
        S *= 2
    if S == 1:
        dw = torch.matmul(dy.t(), x).float()
        return step_blocked_rows(dw, blocked_d, inverse=True) if blocked_d else dw
    part = torch.bmm(dy.view(S, M // S, N).transpose(1, 2), x.view(S, M // S, K))
    # fp32 sum over the S partials; with blocked rows the sum's output order un-permutes them
    perm = (blocked_d // 64, 7) if blocked_d else (1, 1)
    return colsum(part.view(S, N * K), perm).view(N, K)


def wgrad_mfma_slabs(dy, x):
    """The split-L MFMA weight-gradient kernel alone (sc_gemm_wgrad_bf16: gemm.hip) on the
    current stream: fp32 slabs [S, N, K] whose fixed-order sum is dW = dy^T x, or None when the
    shape is outside the kernel's tiling."""
    M, N = dy.shape
    K = x.shape[1]
    lib = _lib.load()
    S = lib.sc_gemm_wgrad_splits(M, N, K)
    if not S or dy.stride(1) != 1 or x.stride(1) != 1 or dy.stride(0) % 8 or x.stride(0) % 8 \
            or dy.data_ptr() % 16 or x.data_ptr() % 16:
        return None
    part = torch.empty(S, N, K, dtype=torch.float32, device=dy.device)
    rc = lib.sc_gemm_wgrad_bf16(ptr(dy), dy.stride(0), ptr(x), x.stride(0), ptr(part), M, N, K, S,
                                stream_of(dy))
    check(rc, "sc_gemm_wgrad_bf16")
    return part


def wgrad_slab_sum(part, blocked_d=0):
    """dW [N, K] from wgrad_mfma_slabs' slabs: fixed-order sum (sc_colsum), un-permuting
    step-blocked rows when blocked_d = D."""
    S, N, K = part.shape
    perm = (blocked_d // 64, 7) if blocked_d else (1, 1)
    return colsum(part.view(S, N * K), perm).view(N, K)


def wgrad_mfma(dy, x, blocked_d=0):
    """dW = dy^T x in fp32 on the MFMA split-L kernel (sc_gemm_wgrad_bf16: gemm.hip) plus the
    fixed-order slab sum (sc_colsum, which also un-permutes step-blocked rows), or None when the
    shape is outside the kernel's tiling (the caller uses the library GEMM)."""
    part = wgrad_mfma_slabs(dy, x)
    return None if part is None else wgrad_slab_sum(part, blocked_d)


# SC_WGRAD_STREAM=1 (A/B only): a cell's weight-gradient kernel on a side stream beside the
# input-gradient GEMM, whose 376 tiles of 256 x 256 fill 1.5 waves of the 256 CUs, so that the
# weight gradient's workgroups take the CUs its last wave leaves idle (slab sum and everything
# after on the main stream; bitwise the same results).  Measured slower at C2 (5.13 vs 5.04 ms
# per step): the persistent weight-gradient workgroups, started piecemeal, lose the per-XCD L2
# sharing of their L-split (268 vs 165 us) and the library GEMM gets no faster.  Default off.
USE_WGRAD_STREAM = os.environ.get("SC_WGRAD_STREAM", "0") == "1"
_SIDE_STREAMS = {}


def _side_stream(dev):
    s = _SIDE_STREAMS.get(dev)
    if s is None:
        s = _SIDE_STREAMS[dev] = torch.cuda.Stream(device=dev)
    return s


# SC_WGRAD128=1: layer 0's weight gradient on the MFMA kernel's 128-column tile over a
# zero-padded copy of its 80 features (fp32 dW, 4.6e-7 of fp32 against the library's bf16 dW at
# 2.6e-3).  Opt-in: same-box A/B 5.200-5.265 ms/step on vs 5.178-5.192 off (profiles/r6f_wgrad128_ab.md)
USE_WGRAD128 = os.environ.get("SC_WGRAD128", "0") != "0"

# SC_TN=0 routes the projection GEMMs back to the library (A/B timing in tools/ only)
USE_TN = os.environ.get("SC_TN", "1") != "0"


def tn_ok(a, b):
    """True when C = a b^T runs on the hand-written MFMA kernel (sc_gemm_tn_bf16): bf16 ROCm
    operands, K-contiguous, K % 64 == 0, N % 256 == 0, 16-byte aligned rows."""
    return (USE_TN and a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16
            and a.dim() == 2 and b.dim() == 2 and a.shape[1] == b.shape[1]
            and a.shape[1] % 64 == 0 and b.shape[0] % 256 == 0 and a.shape[0] > 0
            and a.stride(1) == 1 and b.stride(1) == 1 and a.stride(0) % 8 == 0
            and b.stride(0) % 8 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0
            and (a.shape[0] + 256) * max(a.stride(0), b.shape[0]) * 2 < 2 ** 32
            and b.shape[0] * b.stride(0) * 2 < 2 ** 32)


# SC_TN_FWD=<tile_m>: the K = 512 forward projections on sc_gemm_tn_bf16 with that tile code
# (A/B of the hand-written kernels against the library in the step; default: the library)
TN_FWD_TILE = int(os.environ.get("SC_TN_FWD", "-1"))


def proj_fwd(x, w):
    """x [M,K] @ w [N,K]^T for the frame-major projections.  Measured at the C2 shapes
    (tools/tn_bench.py): the hand-written kernel wins where the output stream dominates (layer 0,
    K = 80 padded to 128: 116 vs 128 us); at K = 512 the library's 256 x 192 tiles win (157 vs
    246 us; csrc/tn_gemm.hip header)."""
    if x.shape[1] <= 128 and tn_ok(x, w):
        return gemm_tn(x, w, 256)   # 256 x 256 four-phase kernel: 114 us vs 120 (192-row tiles)
    if TN_FWD_TILE >= 0 and tn_ok(x, w):
        return gemm_tn(x, w, TN_FWD_TILE)
    return torch.matmul(x, w.t())


def proj_dgrad(dy, w):
    """dy [M,N] @ w [N,K] as dy (w^T)^T: the library's NT kernels beat its NN choice for these
    shapes (gate input gradient 142 vs 160 us; output projection 52 vs 143 us in-step with the
    stream-K kernel the NN form picks); w^T is a 3.7 MB / 1 MB copy."""
    wt = w.t().contiguous()
    return torch.matmul(dy, wt.t())


def gemm_tn(a, b, tile_m=0):
    """C [M,N] bf16 = a [M,K] b [N,K]^T on the persistent MFMA kernel (csrc/tn_gemm.hip);
    the caller checks tn_ok(a, b)."""
    M, K = a.shape
    N = b.shape[0]
    c = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    rc = _lib.load().sc_gemm_tn_bf16(ptr(a), a.stride(0), ptr(b), b.stride(0), ptr(c), c.stride(0),
                                     M, N, K, tile_m, stream_of(a))
    check(rc, "sc_gemm_tn_bf16")
    return c


def pad_cols(x, k, dtype):
    """x [M, K0] -> [M, k] in `dtype` with zero columns K0..k-1 (one cast-copy + one fill)."""
    M, k0 = x.shape
    out = torch.empty(M, k, dtype=dtype, device=x.device)
    out[:, k0:].zero_()
    out[:, :k0].copy_(x)
    return out


# bf16 images of fp32 weights, per parameter: (key, (img, img_t)).  Rebuilt only when the
# parameter changed (its version counter moves with every in-place update: torch's optimizers,
# optim.clip_and_adam_step, load_state_dict) -- so once per optimizer step, in ONE launch for all
# the weights of a model.
from torch.utils.weak import WeakIdKeyDictionary  # noqa: E402

_IMAGES = WeakIdKeyDictionary()
# STATECATCHER_CHECK_IMAGES=1: on every cache hit, compare a few elements of the image with the
# weight (one host sync per weight; a debugging aid for writes that bypass the version counter)
_CHECK_IMAGES = os.environ.get("STATECATCHER_CHECK_IMAGES", "0") == "1"


def invalidate_weight_images(params=None):
    """Drop the cached bf16 images (of ``params``, or of every weight).  Needed only after a
    write that bypasses the parameter's version counter -- ``p.data.copy_(...)`` or
    ``p.data = ...`` (e.g. an EMA / averaged-weight swap): in-place updates through the parameter
    itself (optimizers, ``load_state_dict``, ``with torch.no_grad(): p.copy_(...)``) are seen."""
    if params is None:
        _IMAGES.clear()
        _FOLD.clear()
        _SPLIT_W.clear()
        return
    for p in params:
        _IMAGES.pop(p, None)
        _FOLD.pop(p, None)
        _SPLIT_W.pop(p, None)


def _image_stale(w, img):
    """Debug check: the first / last element of the image against the weight's bf16 value."""
    flat = w.detach().reshape(-1)
    probe = torch.stack([flat[0], flat[-1]]).to(torch.bfloat16).float()
    return not torch.equal(probe, torch.stack([img.reshape(-1)[0], img.reshape(-1)[-1]]).float()) \
        if img.dim() == 1 or img.shape[-1] == w.shape[-1] else False


def weight_images(specs):
    """specs: [(w, block_d, cols_pad, want_t)] with w fp32 [rows, cols] (or [cols]) on the GPU.
    Returns [(img bf16 [rows, cols_pad] (step-blocked rows when block_d), img_t bf16 [cols, rows]
    or None)], reusing cached images of unchanged weights; stale ones are rebuilt together by
    sc_weight_images (csrc/optim.hip)."""
    out, jobs, keep = [None] * len(specs), [], []
    for i, (w, bd, kp, want_t) in enumerate(specs):
        rows, cols = (1, w.shape[0]) if w.dim() == 1 else tuple(w.shape)
        key = (w._version, w.data_ptr(), rows, cols, bd, kp, bool(want_t))
        hit = _IMAGES.get(w)
        if hit is not None and hit[0] == key:
            if _CHECK_IMAGES and bd == 0 and _image_stale(w, hit[1][0]):
                raise RuntimeError("stale bf16 weight image: the weight was written through "
                                   "p.data; call ops.invalidate_weight_images()")
            out[i] = hit[1]
            continue
        img = torch.empty(rows, kp, dtype=torch.bfloat16, device=w.device)
        img_t = torch.empty(cols, rows, dtype=torch.bfloat16, device=w.device) if want_t else None
        ld = w.stride(0) if w.dim() == 2 else cols
        jobs.append(_lib.ImageJob(w.data_ptr(), img.data_ptr(),
                                  img_t.data_ptr() if img_t is not None else None,
                                  rows, cols, kp, ld, bd))
        keep.append(w)
        out[i] = (img.view(-1) if w.dim() == 1 else img, img_t)
        _IMAGES[w] = (key, out[i])
    if jobs:
        _image_jobs(jobs, keep)
    return out


def _image_jobs(jobs, keep):
    require_device(*keep)
    lib = _lib.load()
    for k in range(0, len(jobs), 16):
        part = jobs[k:k + 16]
        rc = lib.sc_weight_images((_lib.ImageJob * len(part))(*part), len(part),
                                  stream_of(keep[0]))
        check(rc, "sc_weight_images")


def cast_pad_bf16(x, kp):
    """fp32 x [M, K] (unit column stride) -> (bf16 [M, kp] with zero columns K..kp-1, bf16
    [M, K]) in one sc_weight_images launch: layer 0's GEMM operand (K padded to the TN kernel's
    stage) and the weight gradient's unpadded copy, instead of a fill, a cast-copy and a cast."""
    M, K = x.shape
    xg = torch.empty(M, kp, dtype=torch.bfloat16, device=x.device)
    xc = torch.empty(M, K, dtype=torch.bfloat16, device=x.device)
    jobs = [_lib.ImageJob(x.data_ptr(), xg.data_ptr(), None, M, K, kp, x.stride(0), 0),
            _lib.ImageJob(x.data_ptr(), xc.data_ptr(), None, M, K, K, x.stride(0), 0)]
    _image_jobs(jobs, [x])
    return xg, xc


def cell_image_spec(w, cdt, needs_dx):
    """The weight image LucyCellFn consumes for w [7D, Din] under compute dtype cdt:
    (w, block_d, cols_pad, want_t), or None when the cell casts w itself (not bf16 / not a
    64-multiple D)."""
    D = w.shape[0] // 7
    if not (cdt == torch.bfloat16 and w.is_cuda and w.dtype == torch.float32 and w.dim() == 2
            and w.stride(1) == 1 and D % 64 == 0):
        return None
    Din = w.shape[1]
    kp = Din + (-Din) % 64
    tn = USE_TN and (7 * D) % 256 == 0
    return (w, D, kp if tn else Din, needs_dx)


def step_blocked_rows(w, D, inverse=False, dtype=None):
    """Permute the 7*D rows of a gate projection weight from the reference's (gate, unit) order
    to (column block of 64 units, gate, unit-in-block) order (inverse=True: back), converting to
    `dtype` in the same copy."""
    K = w.shape[1]
    v = w.view(D // 64, 7, 64, K) if inverse else w.view(7, D // 64, 64, K)
    out = torch.empty((v.shape[1], v.shape[0], 64, K), dtype=dtype or w.dtype, device=w.device)
    out.copy_(v.transpose(0, 1))
    return out.view(7 * D, K)


class LucyCellFn(torch.autograd.Function):
    """One LucyRNN layer: gates = x W^T (one GEMM, compute dtype `cdt`) -> HIP scan, which adds
    the fp32 bias b to the gates on load (a bias epilogue costs the GEMM ~25%, measured).
    Returns (out [B,T,D] in cdt, s_last fp32, h_last fp32): h_last is out[:, -1] before the
    output rounding, the state the next segment starts from (the reference carries out[:, -1]
    in x.dtype, fp32, lucyrnn_triton.py:58/135).

    Backward: scan adjoint (which also emits the bias gradient as per-row partial sums),
    dx = dgates W, dW = split-K dgates^T x.  lucyrnn_triton.py:50-75 fused into one node.
    """

    @staticmethod
    def forward(ctx, x2d, w, b, h0, s0, B, T, cdt, imgs=None, split_sink=None, rec_sink=None):
        """split_sink: a list; when given (bf16), the scan also writes the split-precision planes
        of its output (sc_lucy_scan_fwd_split) and the [B,T,3D] buffer is appended to it (out is
        its first D columns): the input of CTCHeadFn's one-GEMM fp32-accurate projection.
        rec_sink: a list; when given, the scan also writes its output's LayerNorm block records
        (sc_lucy_scan_fwd_ln) for the next layer's LucyCellLNFn, appended to it."""
        ctx.set_materialize_grads(False)   # unused state outputs: no zero-filled gradients
        D = w.shape[0] // 7
        blocked = D % 64 == 0
        Din = x2d.shape[1]
        # layer 0 (Din = 80): the bf16 cast writes zero columns up to a multiple of 64, the
        # MFMA kernel's K stage (the weight gets the same zero columns)
        kp = Din + (-Din) % 64
        tn = USE_TN and x2d.is_cuda and cdt == torch.bfloat16 and (7 * D) % 256 == 0
        # the forward GEMM's copy of x with zero columns up to kp; the weight gradient keeps the
        # unpadded xc (its GEMM would otherwise sum 48 extra zero columns)
        if tn and kp != Din and x2d.dtype == torch.float32 and x2d.stride(1) == 1:
            xg, xc = cast_pad_bf16(x2d, kp)
        else:
            xc = x2d.to(cdt)
            xg = pad_cols(x2d, kp, cdt) if tn and kp != Din else xc
        wt = None
        if imgs is not None:
            # images from weight_images (cell_image_spec): the step-blocked, zero-padded bf16
            # weight and its unpadded transpose for the input gradient
            wg, wt = imgs
            wc = None
            if wt is None and ctx.needs_input_grad[0]:
                wt = step_blocked_rows(w, D, dtype=cdt).t().contiguous()
        else:
            # step-blocked gates: weight rows permuted to (column block, gate, unit) order so
            # each step's 7 x 64 gates of a column block are one contiguous 896-byte run
            wc = step_blocked_rows(w, D, dtype=cdt) if blocked else w.to(cdt)
            wg = pad_cols(wc, kp, cdt) if tn and kp != Din else wc
        bias = b.detach().to(torch.float32).contiguous()
        with _timed("gate_gemm_fwd", xc, 0):
            gates = proj_fwd(xg, wg)
        gates = gates.view(B, T, D // 64, 7, 64) if blocked else gates.view(B, T, 7, D)
        need = any(ctx.needs_input_grad)
        rec = None
        if rec_sink is not None:
            rec = torch.empty(B, T, D // 64, 2, dtype=torch.float32, device=gates.device)
            rec_sink.append(rec)
        res = _scan_fwd(gates, h0, s0, need, bias, want_h=True, split=split_sink is not None,
                        ln=None if rec is None else (None, None, None, rec, 0.0))
        gates, out, s_out, ckpt, h_out = res[:5]
        if len(res) > 5:
            split_sink.append(res[5])
        if need:
            # layer 0 (Din = 80): the weight gradient runs on the MFMA kernel's 128-column tile over
            # the zero-padded copy (sc_gemm_wgrad_bf16, J = 128), and dW keeps the first Din columns
            xw = xg if (USE_WGRAD128 and xg is not xc and xg.shape[1] % 128 == 0
                        and xg.shape[1] % 256 and ctx.needs_input_grad[1]) else xc
            ctx.save_for_backward(xw, wc, wt, gates, ckpt, bias)
            ctx.dtypes = (x2d.dtype, w.dtype, h0.dtype, s0.dtype)
            ctx.blocked = blocked
            ctx.din = Din
        return out, s_out, h_out

    @staticmethod
    def backward(ctx, dout, ds_last, dh_last):
        xc, wc, wt, gates, ckpt, bias = ctx.saved_tensors
        xdt, wdt, hdt, sdt = ctx.dtypes
        if dh_last is not None:   # h_last is out[:, -1]: its gradient joins dout's last step
            B, T = gates.shape[:2]
            if dout is None:
                dout = torch.zeros(B, T, dh_last.shape[-1], dtype=gates.dtype, device=gates.device)
            else:
                dout = dout.clone()
            dout[:, -1] += dh_last.to(dout.dtype)
        dgates, dh0, ds0, dbias = _scan_bwd(gates, ckpt, dout, ds_last, ctx.needs_input_grad[2],
                                            bias)
        dg2 = dgates.view(xc.shape[0], -1)
        bd = (dg2.shape[1] // 7) if ctx.blocked else 0
        # the weight gradient's MFMA kernel on the side stream, beside the input gradient
        part = None
        if (USE_WGRAD_STREAM and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]
                and dg2.is_cuda and dg2.dtype == torch.bfloat16 and xc.dtype == torch.bfloat16):
            main = torch.cuda.current_stream(dg2.device)
            side = _side_stream(dg2.device)
            side.wait_stream(main)   # dgates and x are complete
            with torch.cuda.stream(side):
                with _timed("gate_gemm_wgrad", dg2, 0):
                    part = wgrad_mfma_slabs(dg2, xc)
            if part is not None:
                # (allocator: their blocks are not reused before the side stream's reads end)
                dg2.record_stream(side)
                xc.record_stream(side)
        dx = None
        if ctx.needs_input_grad[0]:
            with _timed("gate_gemm_dgrad", dg2, 0):
                dx = torch.matmul(dg2, wt.t()) if wt is not None else proj_dgrad(dg2, wc)
            dx = dx.to(xdt)
        dw = None
        if part is not None:
            main.wait_stream(side)
            part.record_stream(main)
            dw = wgrad_slab_sum(part, bd)
            if dw.shape[1] != ctx.din:   # (the zero-padded columns of layer 0's copy)
                dw = dw[:, :ctx.din].contiguous()
            dw = dw.to(wdt)
        elif ctx.needs_input_grad[1]:
            with _timed("gate_gemm_wgrad", dg2, 0):
                dw = wgrad_splitk(dg2, xc, blocked_d=bd)
            if dw.shape[1] != ctx.din:   # (the zero-padded columns of layer 0's copy)
                dw = dw[:, :ctx.din].contiguous()
            dw = dw.to(wdt)
        db = colsum(dbias.view(dbias.shape[0], -1)).to(wdt) if dbias is not None else None
        return dx, dw, db, dh0.to(hdt), ds0.to(sdt), None, None, None, None, None, None


def lucy_cell(x, w, b, h0, s0, cdt=None, imgs=None, split_sink=None, rec_sink=None):
    """x [B,T,Din] -> (out [B,T,D], s_last [B,D] fp32, h_last [B,D] fp32) through projection
    + scan.  imgs: the (forward weight, transposed weight) images of cell_image_spec, or None
    (the cell casts w itself).  split_sink: see LucyCellFn.forward."""
    B, T, Din = x.shape
    if cdt is None:
        cdt = torch.promote_types(x.dtype, w.dtype)
    return LucyCellFn.apply(x.reshape(B * T, Din), w, b, h0, s0, B, T, cdt, imgs, split_sink,
                            rec_sink)


# ----------------------------------------------------------------------------- LayerNorm fold ---
# SC_LN_FOLD=1 selects the fold (opt-in).  Measured on the C2 step (same box, alternated twice,
# profiles/r5_ln_fold_ab.md): 5.263-5.278 ms folded vs 5.149-5.178 ms unfused.  The fold removes
# ln_fwd / ln_part_sum (~125 us per step) but adds ~14 us of VALU per layer to the scan forward
# (the records and the rstd rebuild) and ~7 us to the scan backward, which are VALU-bound, plus
# the fold's own weight-gradient pieces -- so the LayerNorm kernels stay the default.
# SC_LN_FOLD=2: the fold applied by the gate GEMM itself (sc_gemm_tn_ln_bf16, round 6): the row
# statistics come from the rows as they stream through the GEMM and its epilogue writes the
# normalised gates, so the forward scan is the plain one (no records, no rebuild); the backward
# scan only scales its stored gradient by rstd (sc_lucy_scan_bwd_ln with ln_r = NULL).
LN_FOLD_MODE = int(os.environ.get("SC_LN_FOLD", "0") or 0)
USE_LN_FOLD = LN_FOLD_MODE in (1, 2)
_FOLD = WeakIdKeyDictionary()


def ln_fold_ok(D):
    return USE_LN_FOLD and D in (512, 1024)


def gemm_tn_ln(h2d, wpp, r_img, eps):
    """(gates [M, N] bf16 = rstd (h W''^T - mean r), stat [M, 2] fp32 (rstd, mean)) for the raw
    previous-layer output h2d [M, D] (sc_gemm_tn_ln_bf16)."""
    M, K = h2d.shape
    N = wpp.shape[0]
    c = torch.empty(M, N, dtype=torch.bfloat16, device=h2d.device)
    stat = torch.empty(M, 2, dtype=torch.float32, device=h2d.device)
    rc = _lib.load().sc_gemm_tn_ln_bf16(ptr(h2d), h2d.stride(0), ptr(wpp), wpp.stride(0), ptr(c),
                                        c.stride(0), M, N, K, ptr(r_img), ptr(stat), float(eps),
                                        stream_of(h2d))
    check(rc, "sc_gemm_tn_ln_bf16")
    return c, stat


def fold_images(specs):
    """specs: [(w, b, gamma, beta, block_d, cols_pad, want_t)] of gate projections that follow a
    LayerNorm (gamma, beta).  Returns [(W'' image bf16 [rows, cols_pad] (step-blocked rows),
    W''^T image or None, b' fp32 [rows], r fp32 [rows])] (csrc/ln_fold.hip header), cached per
    weight and rebuilt when any of w, b, gamma, beta changed: one sc_ln_fold_prep launch and one
    sc_weight_images launch for all stale ones."""
    out, preps, jobs, keep = [None] * len(specs), [], [], []
    for i, (w, b, g, be, bd, kp, want_t) in enumerate(specs):
        key = (w._version, w.data_ptr(), b._version, b.data_ptr(), g._version, g.data_ptr(),
               be._version, be.data_ptr(), bd, kp, bool(want_t))
        hit = _FOLD.get(w)
        if hit is not None and hit[0] == key:
            out[i] = hit[1]
            continue
        rows, cols = w.shape
        f32 = dict(dtype=torch.float32, device=w.device)
        shift, bprime, rowsum = (torch.empty(rows, **f32) for _ in range(3))
        preps.append(_lib.LnFoldJob(w.data_ptr(), g.data_ptr(), be.data_ptr(), b.data_ptr(),
                                    shift.data_ptr(), bprime.data_ptr(), rowsum.data_ptr(),
                                    w.stride(0), rows, cols))
        img = torch.empty(rows, kp, dtype=torch.bfloat16, device=w.device)
        img_t = torch.empty(cols, rows, dtype=torch.bfloat16, device=w.device) if want_t else None
        jobs.append(_lib.ImageJob(w.data_ptr(), img.data_ptr(),
                                  img_t.data_ptr() if img_t is not None else None, rows, cols, kp,
                                  w.stride(0), bd, g.data_ptr(), shift.data_ptr()))
        keep += [w, b, g, be, shift]
        # r in the image's (step-blocked) row order, for the GEMM-side fold's epilogue
        r_img = torch.empty_like(rowsum) if bd and rows % (7 * 64) == 0 else None
        out[i] = (img, img_t, bprime, rowsum, r_img if r_img is not None else rowsum)
        _FOLD[w] = (key, out[i])
    if preps:
        require_device(*keep)
        lib = _lib.load()
        for k in range(0, len(preps), 16):
            part = preps[k:k + 16]
            check(lib.sc_ln_fold_prep((_lib.LnFoldJob * len(part))(*part), len(part),
                                      stream_of(keep[0])), "sc_ln_fold_prep")
        _image_jobs(jobs, keep)
        for o in out:   # (new entries) r permuted to the image's row order, after the prep
            if o is not None and o[4] is not o[3]:
                rows = o[3].numel()
                o[4].copy_(o[3].view(7, rows // (7 * 64), 64).transpose(0, 1).reshape(-1))
    return out


def ln_fold_bwd(g, h, stat):
    """dL/dh [M, D] bf16 of the folded LayerNorm's input h from g = dL/du W'' (sc_ln_fold_bwd)."""
    M, D = h.shape
    g = g.contiguous()
    dh = torch.empty_like(h)
    check(_lib.load().sc_ln_fold_bwd(ptr(g), ptr(h), dtype_code(h), ptr(stat), ptr(dh), M, D,
                                     stream_of(h)), "sc_ln_fold_bwd")
    return dh


def ln_fold_wgrad(Mw, w, gamma, beta, dbp):
    """(dW [rows, D], dgamma [D], dbeta [D]) from M = dL/dW'' and dL/db' (sc_ln_fold_wgrad)."""
    rows, D = Mw.shape
    lib = _lib.load()
    dw = torch.empty(rows, D, dtype=torch.float32, device=Mw.device)
    dgb = torch.empty(2, D, dtype=torch.float32, device=Mw.device)
    ws = torch.empty(lib.sc_ln_fold_wgrad_workspace_numel(rows, D), dtype=torch.float32,
                     device=Mw.device)
    g = gamma.detach().contiguous()
    be = beta.detach().contiguous()
    wd = w.detach()
    check(lib.sc_ln_fold_wgrad(ptr(Mw.contiguous()), ptr(wd), wd.stride(0), ptr(g), ptr(be),
                               ptr(dbp.contiguous()), rows, D, ptr(dw), ptr(dgb), ptr(ws),
                               stream_of(Mw)), "sc_ln_fold_wgrad")
    return dw, dgb[0], dgb[1]


class LucyCellLNFn(torch.autograd.Function):
    """LayerNorm(h_prev) (lucyrnn_triton.py:96-97, :136-137) + one LucyRNN layer (LucyCellFn) as
    ONE node, with the LayerNorm folded into the gate projection (csrc/ln_fold.hip): the GEMM
    reads the previous layer's RAW bf16 output against W'' = centred (W diag gamma), and the
    scan rebuilds LN(h) W^T + b as rstd (u - mean r) + b' on load, from the block records the
    previous scan wrote.  No LayerNorm pass in either direction.  bf16 autocast only (the
    weights come from fold_images).

    Backward: the scan's dgates are rstd dL/dgate = dL/du; dL/dh = ln_fold_bwd(dL/du W'');
    dL/dW'' = dgates^T h (split-L MFMA kernel) -> dW, dgamma, dbeta (ln_fold_wgrad); db = the
    scan's dL/db' partial sums."""

    @staticmethod
    def forward(ctx, h2d, w, b, gamma, beta, h0, s0, B, T, fimgs, rec_in, eps, split_sink=None,
                rec_sink=None):
        ctx.set_materialize_grads(False)
        D = w.shape[0] // 7
        wg, wt, bprime, rowsum, r_img = fimgs
        need = any(ctx.needs_input_grad)
        if LN_FOLD_MODE == 2:
            # the GEMM applies the fold (row statistics from the streaming rows), the scan is plain
            with _timed("gate_gemm_fwd", h2d, 0):
                gates, stat = gemm_tn_ln(h2d, wg, r_img, eps)
            gates = gates.view(B, T, D // 64, 7, 64)
            stat = stat.view(B, T, 2)
            res = _scan_fwd(gates, h0, s0, need, bprime, want_h=True, split=split_sink is not None)
            rowsum = None   # (the backward scan: ln_r = NULL, scale only)
        else:
            with _timed("gate_gemm_fwd", h2d, 0):
                gates = proj_fwd(h2d, wg)
            gates = gates.view(B, T, D // 64, 7, 64)
            stat = torch.empty(B, T, 2, dtype=torch.float32, device=h2d.device)
            rec = None
            if rec_sink is not None:
                rec = torch.empty(B, T, D // 64, 2, dtype=torch.float32, device=h2d.device)
                rec_sink.append(rec)
            res = _scan_fwd(gates, h0, s0, need, bprime, want_h=True, split=split_sink is not None,
                            ln=(rowsum, rec_in, stat, rec, eps))
        gates, out, s_out, ckpt, h_out = res[:5]
        if len(res) > 5:
            split_sink.append(res[5])
        if need:
            ctx.save_for_backward(h2d, wt, gates, ckpt, bprime, rowsum, stat, w, gamma, beta)
            ctx.dtypes = (h2d.dtype, w.dtype, h0.dtype, s0.dtype, gamma.dtype, beta.dtype)
        return out, s_out, h_out

    @staticmethod
    def backward(ctx, dout, ds_last, dh_last):
        h2d, wt, gates, ckpt, bprime, rowsum, stat, w, gamma, beta = ctx.saved_tensors
        xdt, wdt, hdt, sdt, gdt, bdt = ctx.dtypes
        if dh_last is not None:   # h_last is out[:, -1]: its gradient joins dout's last step
            B, T = gates.shape[:2]
            if dout is None:
                dout = torch.zeros(B, T, dh_last.shape[-1], dtype=gates.dtype, device=gates.device)
            else:
                dout = dout.clone()
            dout[:, -1] += dh_last.to(dout.dtype)
        need_w = any(ctx.needs_input_grad[1:5])
        dgates, dh0, ds0, dbias = _scan_bwd(gates, ckpt, dout, ds_last, need_w, bprime,
                                            ln=(rowsum, stat))
        dg2 = dgates.view(h2d.shape[0], -1)
        D = h2d.shape[1]
        dh = None
        if ctx.needs_input_grad[0]:
            with _timed("gate_gemm_dgrad", dg2, 0):
                g = torch.matmul(dg2, wt.t())
            dh = ln_fold_bwd(g, h2d, stat.view(-1, 2)).to(xdt)
        dw = db = dgam = dbet = None
        if need_w:
            with _timed("gate_gemm_wgrad", dg2, 0):
                Mw = wgrad_splitk(dg2, h2d, blocked_d=D)
            dbp = colsum(dbias.view(dbias.shape[0], -1))
            dw, dgam, dbet = ln_fold_wgrad(Mw, w, gamma, beta, dbp)
            dw, db, dgam, dbet = dw.to(wdt), dbp.to(wdt), dgam.to(gdt), dbet.to(bdt)
        return (dh, dw, db, dgam, dbet, dh0.to(hdt), ds0.to(sdt), None, None, None, None, None,
                None, None)


def lucy_cell_ln(h, w, b, gamma, beta, h0, s0, fimgs, rec_in, eps, split_sink=None, rec_sink=None):
    """h [B,T,D] bf16 (the previous layer's raw output) -> (out, s_last, h_last) of
    LayerNorm(gamma, beta, eps) + the cell (w, b), folded (LucyCellLNFn)."""
    B, T, D = h.shape
    h2 = h.reshape(B * T, D)
    if not h2.is_contiguous() or h2.data_ptr() % 16:
        h2 = h2.contiguous()
    return LucyCellLNFn.apply(h2, w, b, gamma, beta, h0, s0, B, T, fimgs, rec_in, eps,
                              split_sink, rec_sink)


# ----------------------------------------------------------------------------- LayerNorm -----
class LayerNormFn(torch.autograd.Function):
    """nn.LayerNorm over the last dim in x's dtype with fp32 statistics (layernorm.hip)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, eps):
        require_device(x)
        D = x.shape[-1]
        x2 = x.reshape(-1, D)
        if not x2.is_contiguous() or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        rows = x2.shape[0]
        g = gamma.detach().to(torch.float32).contiguous()
        b = beta.detach().to(torch.float32).contiguous()
        y = torch.empty_like(x2)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        rc = _lib.load().sc_layernorm_fwd(ptr(x2), dtype_code(x2), ptr(g), ptr(b), ptr(y), ptr(mean),
                                          ptr(rstd), rows, D, float(eps), stream_of(x2))
        check(rc, "sc_layernorm_fwd")
        ctx.save_for_backward(x2, g, mean, rstd)
        ctx.pdtypes = (gamma.dtype, beta.dtype)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, g, mean, rstd = ctx.saved_tensors
        rows, D = x2.shape
        dy2 = dy.reshape(rows, D).to(x2.dtype)
        if not dy2.is_contiguous() or dy2.data_ptr() % 16:
            dy2 = dy2.contiguous()
        lib = _lib.load()
        dx = torch.empty_like(x2)
        dgb = torch.empty(2, D, dtype=torch.float32, device=x2.device)
        ws = torch.empty(lib.sc_layernorm_bwd_workspace_numel(rows, D), dtype=torch.float32,
                         device=x2.device)
        rc = lib.sc_layernorm_bwd(ptr(x2), ptr(dy2), dtype_code(x2), ptr(g), ptr(mean), ptr(rstd),
                                  ptr(dx), ptr(dgb), ptr(ws), rows, D, stream_of(x2))
        check(rc, "sc_layernorm_bwd")
        gd, bd = ctx.pdtypes
        return dx.view(dy.shape), dgb[0].to(gd), dgb[1].to(bd), None


def layer_norm(x, gamma, beta, eps=1e-5):
    return LayerNormFn.apply(x, gamma, beta, eps)


def layer_norm_supported(x):
    return x.dtype in _lib._DTYPE and bool(_lib.load().sc_layernorm_supported(dtype_code(x), x.shape[-1]))


# ----------------------------------------------------------------------------- decay scan ----
class DecayScanFn(torch.autograd.Function):
    """s_t = decay_t * s_{t-1} + kv_t, s_{-1} = init (zeros if None).  lucyrnn_triton.py:158-177."""

    @staticmethod
    def forward(ctx, kv, decay, init):
        require_device(kv, decay, init)
        if kv.shape != decay.shape or kv.dim() != 3:
            raise ValueError(f"kv/decay must be equal [B,T,D]; got {tuple(kv.shape)}, {tuple(decay.shape)}")
        decay = decay.to(kv.dtype)
        kv = kv.contiguous()
        decay = decay.contiguous()
        B, T, D = kv.shape
        initc = None if init is None else init.detach().to(torch.float32).contiguous()
        out = torch.empty_like(kv)
        rc = _lib.load().sc_decay_scan_fwd(ptr(kv), ptr(decay), ptr(out), dtype_code(kv), ptr(initc),
                                           B, T, D, kv.stride(0), kv.stride(1), 1, stream_of(kv))
        check(rc, "sc_decay_scan_fwd")
        ctx.save_for_backward(decay, out, initc)
        ctx.has_init = init is not None
        ctx.init_dtype = None if init is None else init.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        decay, s_all, initc = ctx.saved_tensors
        B, T, D = decay.shape
        dout = dout.to(decay.dtype).contiguous()
        dkv = torch.empty_like(decay)
        ddec = torch.empty_like(decay)
        dinit = torch.zeros(B, D, dtype=torch.float32, device=decay.device) if ctx.has_init else None
        rc = _lib.load().sc_decay_scan_bwd(ptr(decay), ptr(s_all), ptr(dout), ptr(dkv), ptr(ddec),
                                           dtype_code(decay), ptr(initc),
                                           ptr(dinit) if T > 0 else None, B, T, D,
                                           decay.stride(0), decay.stride(1), 1, stream_of(decay))
        check(rc, "sc_decay_scan_bwd")
        return dkv, ddec, (dinit.to(ctx.init_dtype) if ctx.has_init else None)


def decay_scan(kv, decay, init=None):
    return DecayScanFn.apply(kv, decay, init)


# ----------------------------------------------------------------------------- CTC -----------
def _as_len_tensor(x, device):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=torch.int64).contiguous()
    return torch.as_tensor(list(x), dtype=torch.int64).to(device, non_blocking=True)


class CTCFn(torch.autograd.Function):
    """nll [B] fp32 of CTC over x [B,T,V] (logits with fused log_softmax, or log-probs)."""

    @staticmethod
    def forward(ctx, x, targets, in_lens, tgt_lens, blank, is_logits, ex=None):
        """ex: optional fp32 [B, T, U_max + 1] exact emission logits (blank, then each label;
        sc_ctc_fwd_ex), read instead of x's values at those columns."""
        require_device(x, targets, in_lens, tgt_lens)
        if x.dim() != 3:
            raise ValueError(f"x must be [B,T,V], got {tuple(x.shape)}")
        B, T, V = x.shape
        if x.stride(2) != 1:
            x = x.contiguous()
        if targets.dim() != 2 or targets.shape[0] != B:
            raise ValueError("targets must be padded [B, U_max] (the layout train.py:208 builds); "
                             f"got {tuple(targets.shape)}")
        targets = targets.to(torch.int64).contiguous()
        umax = targets.shape[1]
        nll = torch.empty(B, dtype=torch.float32, device=x.device)
        lib = _lib.load()
        wsb = lib.sc_ctc_workspace_bytes(B, max(T, 1), umax)
        ws = torch.empty(wsb, dtype=torch.uint8, device=x.device)
        if ex is not None:
            require_device(x, ex)
            if (ex.dtype != torch.float32 or ex.shape != (B, T, umax + 1) or ex.stride(2) != 1):
                raise ValueError(f"ex must be fp32 [B, T, U_max + 1] = {(B, T, umax + 1)} with unit "
                                 f"column stride; got {ex.dtype} {tuple(ex.shape)}")
        if T == 0:
            nll = torch.where(tgt_lens == 0, 0.0, float("inf")).to(torch.float32)
        else:
            rc = lib.sc_ctc_fwd_ex(ptr(x), dtype_code(x), int(is_logits), B, T, V, x.stride(0),
                                   x.stride(1), ptr(targets), targets.stride(0) if umax else 0, umax,
                                   ptr(in_lens), ptr(tgt_lens), blank, ptr(ex),
                                   ex.stride(0) if ex is not None else 0,
                                   ex.stride(1) if ex is not None else 0, ptr(nll), ptr(ws), wsb,
                                   stream_of(x))
            check(rc, "sc_ctc_fwd_ex")
        ctx.save_for_backward(x, targets, in_lens, tgt_lens, nll, ws)
        ctx.meta = (blank, int(is_logits), umax, wsb)
        ctx.ex = ex
        return nll

    @staticmethod
    def _bwd(ctx, x, targets, in_lens, tgt_lens, nll, ws, scale, grad):
        blank, is_logits, umax, wsb = ctx.meta
        B, T, V = x.shape
        ex = ctx.ex
        rc = _lib.load().sc_ctc_bwd_ex(ptr(x), dtype_code(x), is_logits, B, T, V, x.stride(0),
                                       x.stride(1), ptr(targets), targets.stride(0) if umax else 0,
                                       umax, ptr(in_lens), ptr(tgt_lens), blank, ptr(ex),
                                       ex.stride(0) if ex is not None else 0,
                                       ex.stride(1) if ex is not None else 0, ptr(nll), ptr(scale),
                                       ptr(grad), dtype_code(grad), ptr(ws), wsb, stream_of(x))
        check(rc, "sc_ctc_bwd_ex")

    @staticmethod
    def backward(ctx, grad_nll):
        x, targets, in_lens, tgt_lens, nll, ws = ctx.saved_tensors
        blank, is_logits, umax, wsb = ctx.meta
        B, T, V = x.shape
        grad = torch.empty(B, T, V, dtype=x.dtype, device=x.device)
        if T > 0:
            scale = grad_nll.to(torch.float32).contiguous()
            CTCFn._bwd(ctx, x, targets, in_lens, tgt_lens, nll, ws, scale, grad)
        return grad, None, None, None, None, None, None


class CTCMeanFn(torch.autograd.Function):
    """nn.CTCLoss(reduction='mean', zero_infinity=True) as one autograd node: the lattice
    (sc_ctc_fwd), the reduction and its per-sequence gradient factors (sc_ctc_mean) in the
    forward; the backward is one scale (factor x upstream gradient) and sc_ctc_bwd."""

    @staticmethod
    def forward(ctx, x, targets, in_lens, tgt_lens, blank, is_logits, ex=None):
        nll = CTCFn.forward(ctx, x, targets, in_lens, tgt_lens, blank, is_logits, ex)
        B = nll.shape[0]
        loss = torch.empty((), dtype=torch.float32, device=x.device)
        factor = torch.empty(B, dtype=torch.float32, device=x.device)
        if B:
            rc = _lib.load().sc_ctc_mean(ptr(nll), ptr(tgt_lens), B, ptr(loss), ptr(factor),
                                         stream_of(x))
            check(rc, "sc_ctc_mean")
        else:
            loss.fill_(float("nan"))   # mean over an empty batch
        ctx.factor = factor
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        return CTCFn.backward(ctx, ctx.factor * grad_loss)


def _logits_fp32(x2, wc, b):
    """x2 [M,K] bf16 @ wc [V,K]^T + b (fp32) -> fp32 [M,V]: the MFMA accumulator leaves the GEMM
    unrounded (hipBLASLt with an fp32 D)."""
    return torch.addmm(b, x2, wc.t(), out_dtype=torch.float32)


_SPLIT_W = WeakIdKeyDictionary()

# CTCHeadFn with the scan's split planes:
#   "emis" (default) = the bf16 GEMM's bf16 logits, plus the columns the lattice reads as
#          emissions (blank and each sequence's labels) computed to fp32 accuracy into a
#          [B, T, U + 1] side array that sc_ctc_fwd_ex / _bwd_ex read instead of those columns;
#   "labels" = fp32 logits from the bf16 GEMM with the emission columns scattered in;
#   "full" = every logit from the split-precision GEMM (3x the flops).
# All three give the fp32 oracle's gradients (cosine 1.0000, tools/bf16_logits_diag.py
# "round+exact"): the CTC gradient's sensitivity to the logits is in the lattice's emissions; the
# other columns enter only through the row's log-sum-exp (a per-frame shift every path shares)
# and the softmax term, where bf16 rounding is noise-sized.
# In "emis" the reported loss takes each row's log-sum-exp over the bf16 logits while the
# emission numerators are the side array's exact values: the loss VALUE differs from an fp32 head
# by a per-frame offset of bf16-rounding size (the gradient is unaffected: the lse enters it only
# through the softmax term).
HEAD_SPLIT = os.environ.get("SC_HEAD_SPLIT", "emis")
if HEAD_SPLIT not in ("emis", "labels", "full"):
    raise ValueError(f"SC_HEAD_SPLIT={HEAD_SPLIT!r}: expected 'emis', 'labels' or 'full'")


def _emission_logits(wide, w, b, targets, blank, V):
    """fp32 [B, T, U + 1]: x.W + b at the blank and at each sequence's label columns, to fp32
    accuracy from the scan's [x_hi | x_hi | x_lo] planes: one batched bf16 GEMM against the
    [W_hi | W_lo | W_hi] rows of those columns (K = 3D, fp32 out), gathered and split in one
    launch (sc_ctc_split_rows)."""
    B, T, K3 = wide.shape
    K = K3 // 3
    U1 = targets.shape[1] + 1
    wg = torch.empty(B, U1, K3, dtype=torch.bfloat16, device=wide.device)   # [B, U + 1, 3D]
    bg = torch.empty(B, U1, dtype=torch.float32, device=wide.device)
    tgc = targets.to(torch.int64).contiguous()
    wc_ = w.detach().contiguous()
    rc = _lib.load().sc_ctc_split_rows(ptr(wc_), wc_.stride(0), ptr(b.detach().contiguous()), V, K,
                                       ptr(tgc), tgc.stride(0) if U1 > 1 else 0, U1 - 1, blank,
                                       ptr(wg), ptr(bg), B, stream_of(wide))
    check(rc, "sc_ctc_split_rows")
    ex = torch.bmm(wide, wg.transpose(1, 2), out_dtype=torch.float32)
    ex += bg.unsqueeze(1)
    return ex


def _emission_columns(targets, blank, V):
    """[B, U + 1] column index of _emission_logits' entries (blank, then each label)."""
    B = targets.shape[0]
    return torch.cat([torch.full((B, 1), blank, dtype=torch.int64, device=targets.device),
                      targets.clamp(0, V - 1)], 1)


def _exact_emission_columns(logits, wide, w, b, targets, blank):
    """logits [B,T,V] fp32 in place: the emission columns set to _emission_logits' values
    (duplicates write equal values)."""
    B, T, V = logits.shape
    ex = _emission_logits(wide, w, b, targets, blank, V)
    lab = _emission_columns(targets, blank, V)
    logits.scatter_(2, lab.unsqueeze(1).expand(B, T, lab.shape[1]), ex)


def split_weight_image(w):
    """[W_hi | W_lo | W_hi] bf16 [V, 3K] of an fp32 w [V, K] (W_hi = bf16(w), W_lo = bf16(w -
    W_hi)): against [x_hi | x_hi | x_lo] one bf16 GEMM gives x_hi W_hi + x_hi W_lo + x_lo W_hi,
    i.e. x.W to ~2^-16 relative.  Cached per weight version (rebuilt once per optimizer step)."""
    key = (w._version, w.data_ptr(), tuple(w.shape))
    hit = _SPLIT_W.get(w)
    if hit is not None and hit[0] == key:
        return hit[1]
    with torch.no_grad():
        wd = w.detach()
        hi = wd.to(torch.bfloat16)
        lo = (wd - hi.float()).to(torch.bfloat16)
        img = torch.cat([hi, lo, hi], 1)
    _SPLIT_W[w] = (key, img)
    return img


class CTCHeadFn(torch.autograd.Function):
    """output_proj (LinearSafe, lucyrnn_triton.py:107-109, :150) + log_softmax + nn.CTCLoss(
    reduction='mean', zero_infinity=True) (model.py:68-71, train.py:142) as ONE node, for bf16
    autocast training.  Returns (loss, logits).

    Why: rounding the logits to bf16 before the lattice is what costs the bf16 C2 step 2-5% of
    gradient direction against the fp32 oracle (tools/bf16_logits_diag.py reproduces the measured
    cosines from that rounding alone).  Here the projection writes fp32 logits, which the lattice
    reads, and the lattice's gradient is written in bf16 straight into the projection backward's
    operand (a separate fp32 logits tensor would need an fp32 gradient and a cast pass, since
    autograd casts a gradient to its input's dtype).  Under HEAD_SPLIT "emis" (the default) the
    returned logits are the bf16 GEMM's, and only the emission columns reach the lattice at fp32
    accuracy (side array).  The logits output stays differentiable: a
    gradient reaching it from elsewhere is added before the projection backward."""

    @staticmethod
    def forward(ctx, x, w, b, wc, wt, targets, in_lens, tgt_lens, blank, wide=None):
        ctx.set_materialize_grads(False)
        B, T, K = x.shape
        V = w.shape[0]
        x2 = x.reshape(-1, K)
        ex = None
        if wide is not None and HEAD_SPLIT == "full":   # every logit from [x_hi | x_hi | x_lo]
            logits = _logits_fp32(wide.view(-1, 3 * K), split_weight_image(w), b).view(B, T, V)
        elif wide is not None and HEAD_SPLIT == "emis":
            logits = torch.addmm(b.to(torch.bfloat16), x2, wc.t()).view(B, T, V)
            ex = _emission_logits(wide.view(B, T, 3 * K), w, b, targets, blank, V)
        else:
            logits = _logits_fp32(x2, wc, b).view(B, T, V)
            if wide is not None:
                _exact_emission_columns(logits, wide, w, b, targets, blank)
        loss = CTCMeanFn.forward(ctx, logits, targets, in_lens, tgt_lens, blank, True, ex)
        ctx.head = (x2, wt, x.shape, x.dtype)
        return loss, logits

    @staticmethod
    def backward(ctx, g_loss, g_logits):
        logits, targets, in_lens, tgt_lens, nll, ws = ctx.saved_tensors
        blank, is_logits, umax, wsb = ctx.meta
        x2, wt, xshape, xdt = ctx.head
        B, T, V = logits.shape
        dy = torch.empty(B, T, V, dtype=torch.bfloat16, device=logits.device)
        if g_loss is None:
            dy.zero_()
        elif T > 0:
            scale = (ctx.factor * g_loss).to(torch.float32).contiguous()
            CTCFn._bwd(ctx, logits, targets, in_lens, tgt_lens, nll, ws, scale, dy)
        if g_logits is not None:
            dy = (dy.float() + g_logits).to(torch.bfloat16)
        dy2 = dy.view(-1, V)
        dx = torch.matmul(dy2, wt.t()).view(xshape).to(xdt) if ctx.needs_input_grad[0] else None
        dw = wgrad_splitk(dy2, x2) if ctx.needs_input_grad[1] else None
        db = colsum(dy2) if ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None, None, None, None, None


def ctc_head_supported(x, w, b, imgs):
    """CTCHeadFn applies: bf16 hidden on the GPU, fp32 projection with a bias, bf16 images of W
    and W^T (LucyRNNtriton._weight_images under bf16 autocast)."""
    return (imgs is not None and imgs[1] is not None and x.is_cuda and x.dtype == torch.bfloat16
            and x.dim() == 3 and b is not None and w.dtype == torch.float32
            and b.dtype == torch.float32)


def ctc_head_loss(x, w, b, imgs, targets, in_lens, tgt_lens, blank=0, wide=None):
    """(loss, logits) of CTCHeadFn -- logits bf16 under SC_HEAD_SPLIT=emis (the default; the
    lattice read its emission columns from the fp32 side array), fp32 under 'labels' / 'full'
    or without `wide`: x [B,T,D] bf16 hidden, w [V,D] / b [V] the fp32
    output_proj parameters, imgs their (W, W^T) bf16 images; wide: the scan's split-precision
    [B,T,3D] buffer whose first D columns are x (LucyCellFn split_sink), or None."""
    dev = x.device
    if wide is not None and not (wide.is_contiguous() and wide.shape[:2] == x.shape[:2]
                                 and wide.shape[2] == 3 * x.shape[2]
                                 and x.data_ptr() == wide.data_ptr()):
        raise ValueError("ctc_head_loss: wide must be the [B,T,3D] buffer x is the head of")
    if wide is None:
        x = x.contiguous()
    return CTCHeadFn.apply(x, w, b, imgs[0], imgs[1], targets.to(dev),
                           _as_len_tensor(in_lens, dev), _as_len_tensor(tgt_lens, dev), int(blank),
                           wide)


def ctc_nll(x, targets, in_lens, tgt_lens, blank=0, is_logits=True):
    dev = x.device
    return CTCFn.apply(x, targets.to(dev), _as_len_tensor(in_lens, dev), _as_len_tensor(tgt_lens, dev),
                       int(blank), bool(is_logits))


def ctc_loss(x, targets, in_lens, tgt_lens, blank=0, reduction="mean", zero_infinity=True,
             is_logits=True):
    """CTC with the semantics of nn.CTCLoss(blank, reduction, zero_infinity) (train.py:142).

    x: [B,T,V]; logits (log_softmax fused, as model.py:70 applies it) or log-probs.
    'mean' = mean_b(nll_b / max(U_b, 1)), 'sum' = sum_b nll_b, 'none' = nll.
    """
    dev = x.device
    tl = _as_len_tensor(tgt_lens, dev)
    if reduction == "mean" and zero_infinity:   # the training criterion (train.py:142): fused
        return CTCMeanFn.apply(x, targets.to(dev), _as_len_tensor(in_lens, dev), tl, int(blank),
                               bool(is_logits))
    nll = CTCFn.apply(x, targets.to(dev), _as_len_tensor(in_lens, dev), tl, int(blank), bool(is_logits))
    if zero_infinity:
        nll = torch.where(torch.isinf(nll), torch.zeros_like(nll), nll)
    if reduction == "none":
        return nll
    if reduction == "sum":
        return nll.sum()
    if reduction == "mean":
        return (nll / tl.clamp_min(1).to(nll.dtype)).mean()
    raise ValueError(f"unknown reduction {reduction!r}")


def ctc_greedy_decode(log_probs, lengths, blank=0):
    """Device greedy decode -> (tokens int32 [B,T], counts int32 [B]) (decoder.py:3-30)."""
    require_device(log_probs)
    B, T, V = log_probs.shape
    if log_probs.stride(2) != 1:
        log_probs = log_probs.contiguous()
    lens = _as_len_tensor(lengths, log_probs.device)
    tokens = torch.empty(B, T, dtype=torch.int32, device=log_probs.device)
    counts = torch.empty(B, dtype=torch.int32, device=log_probs.device)
    rc = _lib.load().sc_ctc_greedy_decode(ptr(log_probs), dtype_code(log_probs), B, T, V,
                                          log_probs.stride(0), log_probs.stride(1), ptr(lens),
                                          int(blank), ptr(tokens), ptr(counts), stream_of(log_probs))
    check(rc, "sc_ctc_greedy_decode")
    return tokens, counts


def ctc_greedy_step(logits, prev, emit, mask=None, blank=0):
    """One streaming frame of decoder.py:3-30 for B streams, in place: logits [B,V] (unit inner
    stride), prev int32 [B] (-1 = stream start), emit int32 view [B] (any stride) <- token or -1.
    mask fp32 [B] or None (0 = frame past the stream's end: emits -1, prev kept)."""
    require_device(logits, prev, emit)
    B, V = logits.shape
    if logits.stride(1) != 1 or prev.dtype != torch.int32 or emit.dtype != torch.int32:
        raise ValueError("ctc_greedy_step: logits need unit inner stride, prev/emit int32")
    if prev.numel() != B or emit.numel() != B or not prev.is_contiguous():
        raise ValueError("ctc_greedy_step: prev/emit must hold B entries (prev contiguous)")
    if mask is not None and (mask.dtype != torch.float32 or mask.numel() != B or mask.stride(0) != 1):
        raise ValueError("ctc_greedy_step: mask must be contiguous fp32 [B]")
    rc = _lib.load().sc_ctc_greedy_step(ptr(logits), dtype_code(logits), B, V, logits.stride(0),
                                        ptr(mask), int(blank), ptr(prev), ptr(emit),
                                        emit.stride(0), stream_of(logits))
    check(rc, "sc_ctc_greedy_step")


# ------------------------------------------------------------------- streaming LucyRNN step --
STEP_FUSED, STEP_UNFUSED_A, STEP_UNFUSED_B = 0, 1, 2


def lucy_step_ln(x, w, b, out, eps=1e-5):
    """out = LayerNorm(x) rows of D (layernorm_in, lucyrnn.py:45), no allocation."""
    B, D = x.shape
    rc = _lib.load().sc_lucy_step_ln(ptr(x), dtype_code(x), ptr(w), ptr(b), float(eps), ptr(out),
                                     B, D, stream_of(x))
    check(rc, "sc_lucy_step_ln")


def lucy_step_cell(mode, g, h, s, out, lnz=None, lnh=None, u=None, hp=None, mask=None, eps=1e-5):
    """One LucyRNNCell step (lucyrnn.py:44-70) on GEMM outputs, state h/s fp32 [B,D] in place
    (include/statecatcher.h sc_lucy_step_cell for the three modes).  lnz/lnh: (weight, bias)
    fp32 or None (layer_norm=False).  No allocation: safe inside a hipGraph capture."""
    B, D = h.shape
    lzw, lzb = lnz if lnz is not None else (None, None)
    lhw, lhb = lnh if lnh is not None else (None, None)
    rc = _lib.load().sc_lucy_step_cell(int(mode), ptr(g), dtype_code(g), g.stride(0), ptr(u),
                                       ptr(hp), ptr(lzw), ptr(lzb), ptr(lhw), ptr(lhb), float(eps),
                                       ptr(h), ptr(s), ptr(out), ptr(mask), B, D, stream_of(g))
    check(rc, "sc_lucy_step_cell")


FRAME_PLAIN, FRAME_STATS, FRAME_CELL_UNFUSED, FRAME_CELL_FUSED = 0, 1, 2, 3


def lucy_frame_gemm(epi, x, w, bias, y, st_out=None, ln=None, st_in=None, z=None, st_z=None,
                    s=None, mask=None, eps=1e-5):
    """One fused GEMM of the streaming frame (csrc/lucy_frame.hip, include/statecatcher.h
    sc_lucy_frame_gemm): x fp32 [B, K] (row stride x.stride(0)), w fp32/bf16 [N, K], bias fp32
    [N], y fp32; ln = (weight, bias) of a LayerNorm prologue over K with st_in its statistics
    records ([n, B, 4] fp32).  No allocation: safe inside a hipGraph capture."""
    B, K = x.shape
    N = w.shape[0]
    lw, lb = ln if ln is not None else (None, None)
    rc = _lib.load().sc_lucy_frame_gemm(
        int(epi), ptr(x), x.stride(0), K, ptr(lw), ptr(lb), ptr(st_in),
        st_in.shape[0] if st_in is not None else 0, float(eps), ptr(w), dtype_code(w), w.stride(0),
        ptr(bias), B, N, ptr(y), y.stride(0), ptr(st_out), ptr(z), ptr(st_z), ptr(s), ptr(mask),
        stream_of(x))
    check(rc, "sc_lucy_frame_gemm")


def lucy_frame_cellb(z, hp, h, out, st_z=None, st_h=None, lnz=None, lnh=None, mask=None, eps=1e-5):
    """h = (1 - sigmoid(LN_z z)) tanh(LN_h hp) + sigmoid(LN_z z) h, masked, in place; out = h
    (sc_lucy_frame_cellb).  lnz / lnh (weight, bias) with their statistics records, or None."""
    B, D = h.shape
    zw, zb = lnz if lnz is not None else (None, None)
    hw, hb = lnh if lnh is not None else (None, None)
    rc = _lib.load().sc_lucy_frame_cellb(
        ptr(z), ptr(st_z), st_z.shape[0] if st_z is not None else 0, ptr(hp), ptr(st_h),
        st_h.shape[0] if st_h is not None else 0, ptr(zw), ptr(zb), ptr(hw), ptr(hb), float(eps),
        ptr(h), ptr(out), out.stride(0), ptr(mask), B, D, stream_of(h))
    check(rc, "sc_lucy_frame_cellb")


def frame_gemm_job(x, w, bias, y, st_out=None, ln=None, st_in=None, z=None, st_z=None, s=None,
                   mask=None):
    """One job of lucy_frame_gemm_multi (the arguments of one lucy_frame_gemm call)."""
    B, K = x.shape
    lw, lb = ln if ln is not None else (None, None)
    return _lib.FrameGemmJob(ptr(x), x.stride(0), K, ptr(lw), ptr(lb), ptr(st_in),
                             st_in.shape[0] if st_in is not None else 0, ptr(w), w.stride(0),
                             ptr(bias), B, w.shape[0], ptr(y), y.stride(0), ptr(st_out), ptr(z),
                             ptr(st_z), ptr(s), ptr(mask))


def lucy_frame_gemm_multi(epi, w_dtype, jobs, stream, eps=1e-5):
    """Independent frame GEMMs of one epilogue kind (FrameGemmJob list, <= 8 per launch: longer
    lists take ceil(n / 8) launches) -- sc_lucy_frame_gemm_multi.  w_dtype: torch dtype of
    every job's weights.  No allocation: safe inside a hipGraph capture."""
    lib = _lib.load()
    code = dtype_code(torch.empty(0, dtype=w_dtype))
    for k in range(0, len(jobs), 8):
        part = jobs[k:k + 8]
        check(lib.sc_lucy_frame_gemm_multi(int(epi), code, float(eps),
                                           (_lib.FrameGemmJob * len(part))(*part), len(part),
                                           stream), "sc_lucy_frame_gemm_multi")


def frame_cell_job(z, hp, h, out, st_z=None, st_h=None, lnz=None, lnh=None, mask=None):
    """One job of lucy_frame_cellb_multi (the arguments of one lucy_frame_cellb call)."""
    B, D = h.shape
    zw, zb = lnz if lnz is not None else (None, None)
    hw, hb = lnh if lnh is not None else (None, None)
    return _lib.FrameCellJob(ptr(z), ptr(st_z), st_z.shape[0] if st_z is not None else 0, ptr(hp),
                             ptr(st_h), st_h.shape[0] if st_h is not None else 0, ptr(zw), ptr(zb),
                             ptr(hw), ptr(hb), ptr(h), ptr(out), out.stride(0), ptr(mask), B, D)


def lucy_frame_cellb_multi(jobs, stream, eps=1e-5):
    """Independent lucy_frame_cellb calls in <= 8-job launches (sc_lucy_frame_cellb_multi)."""
    lib = _lib.load()
    for k in range(0, len(jobs), 8):
        part = jobs[k:k + 8]
        check(lib.sc_lucy_frame_cellb_multi(float(eps), (_lib.FrameCellJob * len(part))(*part),
                                            len(part), stream), "sc_lucy_frame_cellb_multi")


def ctc_greedy_frames(logits, prev, emit, mask=None, blank=0):
    """ctc_greedy_step over F frames in order, one launch (sc_ctc_greedy_frames): logits
    [F, B, V] (unit inner stride), prev int32 [B] contiguous, emit int32 [F, B], mask fp32
    [F, B] (unit inner stride) or None."""
    require_device(logits, prev, emit)
    F, B, V = logits.shape
    if logits.stride(2) != 1 or prev.dtype != torch.int32 or emit.dtype != torch.int32:
        raise ValueError("ctc_greedy_frames: logits need unit inner stride, prev/emit int32")
    if prev.numel() != B or not prev.is_contiguous() or tuple(emit.shape) != (F, B):
        raise ValueError("ctc_greedy_frames: prev [B] contiguous, emit [F, B]")
    if mask is not None and (mask.dtype != torch.float32 or tuple(mask.shape) != (F, B)
                             or mask.stride(1) != 1):
        raise ValueError("ctc_greedy_frames: mask must be fp32 [F, B] with unit inner stride")
    rc = _lib.load().sc_ctc_greedy_frames(
        ptr(logits), dtype_code(logits), F, B, V, logits.stride(0), logits.stride(1), ptr(mask),
        mask.stride(0) if mask is not None else 0, int(blank), ptr(prev), ptr(emit),
        emit.stride(0), emit.stride(1), stream_of(logits))
    check(rc, "sc_ctc_greedy_frames")


# ------------------------------------------------------------------- feature frontend --------
def fbank(audio, kind="mfcc", sample_rate=16000):
    """make_frontend(kind)(audio).transpose(-1, -2) on the GPU (fbank.hip): audio fp32
    [B, N] -> [B, frames, 80] (kind "mfcc" or "mel"; see include/statecatcher.h sc_fbank).
    For "mel", AmplitudeToDB's top_db clamp is relative to the max over the whole call."""
    require_device(audio)
    if audio.dim() != 2:
        raise ValueError(f"fbank: audio must be [B, N], got {tuple(audio.shape)}")
    codes = {"mfcc": 0, "mel": 1}
    if kind not in codes:
        raise ValueError(f"Unsupported frontend: {kind}")
    a = audio.to(torch.float32)
    if a.stride(1) != 1:
        a = a.contiguous()
    lib = _lib.load()
    B, N = a.shape
    F = lib.sc_fbank_frames(N)
    out = torch.empty(B, F, 80, dtype=torch.float32, device=a.device)
    wsb = lib.sc_fbank_workspace_bytes()
    ws = torch.empty(wsb, dtype=torch.uint8, device=a.device)
    rc = lib.sc_fbank(ptr(a), B, N, a.stride(0), codes[kind], float(sample_rate), ptr(out), ptr(ws),
                      wsb, stream_of(a))
    check(rc, "sc_fbank")
    return out


# ----------------------------------------------------------------------------- RNN-T ---------
class RNNTFn(torch.autograd.Function):
    """nll [B] fp32 of the RNN-T lattice (rnnt.hip) over x: dense [B,T,U+1,V] or compact
    [sum_b T_b (U_b+1), V] rows; logits (log_softmax fused) or log-probs."""

    @staticmethod
    def forward(ctx, x, labels, flen, llen, blank, is_logits, row_off, T):
        require_device(x, labels, flen, llen)
        compact = row_off is not None
        if x.stride(-1) != 1:
            x = x.contiguous()
        if compact:
            if x.dim() != 2:
                raise ValueError(f"compact log_probs must be [rows, V], got {tuple(x.shape)}")
            B = flen.shape[0]
            V = x.shape[1]
            sb, st, su = 0, 0, x.stride(0)
        else:
            if x.dim() != 4:
                raise ValueError(f"log_probs must be [B,T,U+1,V], got {tuple(x.shape)}")
            B, T, U1, V = x.shape
            sb, st, su = x.stride(0), x.stride(1), x.stride(2)
        labels = labels.to(torch.int64).contiguous()
        if labels.dim() != 2 or labels.shape[0] != B:
            raise ValueError(f"labels must be padded [B, U_max], got {tuple(labels.shape)}")
        umax = labels.shape[1] if compact else x.shape[2] - 1
        if not compact and labels.shape[1] < umax:
            labels = torch.nn.functional.pad(labels, (0, umax - labels.shape[1]))
        nll = torch.empty(B, dtype=torch.float32, device=x.device)
        lib = _lib.load()
        wsb = lib.sc_rnnt_workspace_bytes(B, max(T, 1), umax)
        ws = torch.empty(wsb, dtype=torch.uint8, device=x.device)
        if T == 0 or B == 0:
            nll.fill_(float("inf"))
        else:
            rc = lib.sc_rnnt_fwd(ptr(x), dtype_code(x), int(is_logits), B, T, umax, V, sb, st, su,
                                 ptr(row_off), ptr(labels), labels.stride(0), ptr(flen), ptr(llen),
                                 blank, ptr(nll), ptr(ws), wsb, stream_of(x))
            check(rc, "sc_rnnt_fwd")
        ctx.save_for_backward(x, labels, flen, llen, ws, row_off)
        ctx.meta = (blank, int(is_logits), umax, wsb, B, T, V, sb, st, su)
        return nll

    @staticmethod
    def backward(ctx, grad_nll):
        x, labels, flen, llen, ws, row_off = ctx.saved_tensors
        blank, is_logits, umax, wsb, B, T, V, sb, st, su = ctx.meta
        grad = torch.empty_like(x, memory_format=torch.contiguous_format)
        if grad.stride() != x.stride():
            raise RuntimeError("rnnt backward expects a contiguous input")
        if T > 0 and B > 0:
            scale = grad_nll.to(torch.float32).contiguous()
            rc = _lib.load().sc_rnnt_bwd(ptr(x), dtype_code(x), is_logits, B, T, umax, V, sb, st, su,
                                         ptr(row_off), ptr(labels), labels.stride(0), ptr(flen),
                                         ptr(llen), blank, ptr(scale), ptr(grad), dtype_code(grad),
                                         ptr(ws), wsb, stream_of(x))
            check(rc, "sc_rnnt_bwd")
        else:
            grad.zero_()
        return grad, None, None, None, None, None, None, None


def rnnt_loss(log_probs, labels, frames_lengths, labels_lengths, average_frames=False,
              reduction="mean", blank=0, gather=False, compact=False, is_logits=False):
    """warp_rnnt.rnnt_loss's interface (model.py:97-105): log_probs [B,T,U+1,V] (or compact
    [sum_b T_b(U_b+1), V]), labels [B,U] int, lengths [B].  reduction 'mean' = mean_b(cost_b),
    'sum', 'none'; average_frames divides each cost by its frame count.  `gather` selects a
    memory strategy in warp_rnnt and does not change the result (the kernels always gather).
    is_logits=True fuses the log_softmax (x are joiner logits)."""
    del gather
    dev = log_probs.device
    fl = _as_len_tensor(frames_lengths, dev)
    ll = _as_len_tensor(labels_lengths, dev)
    row_off = None
    T = 0
    if compact:
        sizes = fl * (ll + 1)
        row_off = torch.cumsum(sizes, 0) - sizes
        T = int(fl.max().item()) if fl.numel() else 0
    nll = RNNTFn.apply(log_probs, labels.to(dev), fl, ll, int(blank), bool(is_logits), row_off, T)
    if average_frames:
        nll = nll / fl.clamp_min(1).to(nll.dtype)
    if reduction == "none":
        return nll
    if reduction == "sum":
        return nll.sum()
    if reduction == "mean":
        return nll.mean()
    raise ValueError(f"unknown reduction {reduction!r}")


class RNNTJointFn(torch.autograd.Function):
    """nll [B] fp32 of the fused joiner + lattice (rnnt.hip joint_* kernels): z = tanh(enc_p[b,t]
    + pred_p[b,u]), logits = z W^T + bias, log_softmax, gathered RNN-T lattice -- the reference's
    RNNTPredictorJoiner (model.py:129-145) + log_softmax (model.py:93) + warp_rnnt, with the
    (B, T, U+1, V) logits never materialised.  enc_p [B,T,64], pred_p [B,U+1,64] are the
    joiner's enc_proj / pred_proj outputs; W [V,64] enters the MFMA in bf16, everything else fp32.
    Backward: d enc_p, d pred_p, dW, d bias (partials summed here in a fixed order)."""

    @staticmethod
    def forward(ctx, enc_p, pred_p, W, bias, labels, flen, llen, blank):
        require_device(enc_p, pred_p, W, bias, labels, flen, llen)
        B, T, J = enc_p.shape
        U1 = pred_p.shape[1]
        Umax = U1 - 1
        V = W.shape[0]
        if pred_p.shape[0] != B or pred_p.shape[2] != J or W.shape[1] != J or bias.shape != (V,):
            raise ValueError(f"joint shapes: enc {tuple(enc_p.shape)} pred {tuple(pred_p.shape)} "
                             f"W {tuple(W.shape)} bias {tuple(bias.shape)}")
        encc = enc_p.detach().float().contiguous()
        predc = pred_p.detach().float().contiguous()
        wb = W.detach().to(torch.bfloat16).contiguous()
        bf = bias.detach().float().contiguous()
        labels = labels.to(torch.int64)
        if labels.dim() != 2 or labels.shape[0] != B:
            raise ValueError(f"labels must be padded [B, U], got {tuple(labels.shape)}")
        if labels.shape[1] < Umax:
            labels = torch.nn.functional.pad(labels, (0, Umax - labels.shape[1]))
        labels = labels[:, :Umax].contiguous()
        lib = _lib.load()
        wsb = lib.sc_rnnt_workspace_bytes(B, max(T, 1), Umax)
        ws = torch.empty(wsb, dtype=torch.uint8, device=enc_p.device)
        nll = torch.empty(B, dtype=torch.float32, device=enc_p.device)
        if T == 0 or B == 0:
            nll.fill_(float("inf"))
        else:
            with _timed("rnnt_joint_fwd", encc, 0):
                rc = lib.sc_rnnt_joint_fwd(ptr(encc), ptr(predc), ptr(wb), ptr(bf), B, T, Umax, V, J,
                                           ptr(labels), labels.stride(0) if Umax else 0, ptr(flen),
                                           ptr(llen), int(blank), ptr(nll), ptr(ws), wsb,
                                           stream_of(encc))
            check(rc, "sc_rnnt_joint_fwd")
        ctx.save_for_backward(encc, predc, wb, bf, labels, flen, llen, ws)
        ctx.meta = (int(blank), wsb, enc_p.dtype, pred_p.dtype, W.dtype, bias.dtype)
        return nll

    @staticmethod
    def backward(ctx, grad_nll):
        encc, predc, wb, bf, labels, flen, llen, ws = ctx.saved_tensors
        blank, wsb, edt, pdt, wdt, bdt = ctx.meta
        B, T, J = encc.shape
        U1 = predc.shape[1]
        Umax = U1 - 1
        V = wb.shape[0]
        dev = encc.device
        if T == 0 or B == 0:
            return (torch.zeros_like(encc).to(edt), torch.zeros_like(predc).to(pdt),
                    torch.zeros(V, J, dtype=wdt, device=dev), torch.zeros(V, dtype=bdt, device=dev),
                    None, None, None, None)
        lib = _lib.load()
        geo = [ctypes_int() for _ in range(3)]
        check(lib.sc_rnnt_joint_geometry(B, T, Umax, V, *[_addr(g) for g in geo]),
              "sc_rnnt_joint_geometry")
        ntb, nus, S = (g.value for g in geo)
        f32 = dict(dtype=torch.float32, device=dev)
        d_enc = torch.empty(nus, B, T, J, **f32)
        d_pred = torch.zeros(B, ntb, U1, J, **f32)
        dW = torch.empty(S, V, J, **f32)
        db = torch.empty(S, V, **f32)
        scale = grad_nll.to(torch.float32).contiguous()
        with _timed("rnnt_joint_bwd", encc, 0):
            rc = lib.sc_rnnt_joint_bwd(ptr(encc), ptr(predc), ptr(wb), ptr(bf), B, T, Umax, V, J,
                                       ptr(labels), labels.stride(0) if Umax else 0, ptr(flen),
                                       ptr(llen), blank, ptr(scale), ptr(d_enc), ptr(d_pred),
                                       ptr(dW), ptr(db), ptr(ws), wsb, stream_of(encc))
        check(rc, "sc_rnnt_joint_bwd")
        # fixed-order sums of the partials (the kernel's dlogits include the sparse blank / label
        # arcs of the gathered lattice)
        dWt = colsum(dW.view(S, V * J)).view(V, J)
        dbt = colsum(db)
        return (d_enc.sum(0).to(edt), d_pred.sum(1).to(pdt), dWt.to(wdt), dbt.to(bdt),
                None, None, None, None)


def ctypes_int():
    import ctypes
    return ctypes.c_int(0)


def _addr(c):
    import ctypes
    return ctypes.addressof(c)


def rnnt_joint_supported(join_dim, vocab):
    """Shapes the fused joiner kernels are compiled for (J = 64, V % 32 == 0, V <= 1024); other
    joiners take the materialised HIP path (logits -> sc_rnnt_*)."""
    return join_dim == 64 and vocab % 32 == 0 and 0 < vocab <= 1024


def rnnt_joint_loss(enc_p, pred_p, W, bias, labels, frames_lengths, labels_lengths, blank=0,
                    reduction="mean", average_frames=False):
    """warp_rnnt's reductions over the fused joiner + lattice (RNNTJointFn)."""
    dev = enc_p.device
    fl = _as_len_tensor(frames_lengths, dev)
    ll = _as_len_tensor(labels_lengths, dev)
    nll = RNNTJointFn.apply(enc_p, pred_p, W, bias, labels.to(dev), fl, ll, int(blank))
    if average_frames:
        nll = nll / fl.clamp_min(1).to(nll.dtype)
    if reduction == "none":
        return nll
    if reduction == "sum":
        return nll.sum()
    if reduction == "mean":
        return nll.mean()
    raise ValueError(f"unknown reduction {reduction!r}")


# ----------------------------------------------------------------------------- mLSTM ---------
_F16_MAX = 65504.0


def _mlstm_fp32_cell(q, k, v):
    """Cell dtype for fp32 q / k / v: f16 (11-bit mantissa, the finer cell) when all three fit
    its range, else bf16 (fp32's range): a magnitude above 65504 would become inf in f16 and NaN
    downstream.  The range check reads one scalar back; inside a HIP-graph capture,
    where it cannot, the range-safe bf16 cell is used."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        return torch.bfloat16
    m = torch.stack([q.abs().amax(), k.abs().amax(), v.abs().amax()]).amax()
    return torch.float16 if bool(m <= _F16_MAX) else torch.bfloat16


class MLSTMFn(torch.autograd.Function):
    """mLSTM cell (mlstm.hip) over q, k [B,NH,T,DQ], v [B,NH,T,DV], gate pre-activations
    [B,NH,T]; returns h [B,NH,T,DV] and the final state (C [B,NH,DQ,DV], n [B,NH,DQ],
    m [B,NH,1]) like transformers' mlstm_chunkwise_native_autograd(return_last_states=True).
    Compute dtype bf16/f16; fp32 inputs are rounded to f16, the finer of the two compiled cells
    (11-bit mantissa; the f16 backward scales its gradients per chunk, so dh below f16's normal
    range is not lost) -- the reference's kernels run under autocast_kernel_dtype = float16
    (model.py:227) -- unless a value exceeds f16's range, then to bf16 (_mlstm_fp32_cell).
    fp32 state."""

    @staticmethod
    def forward(ctx, q, k, v, igate, fgate, c0, n0, m0, eps):
        require_device(q, k, v, igate, fgate)
        ctx.set_materialize_grads(False)   # detached carried states: no zero-filled gradients
        B, NH, T, DQ = q.shape
        DV = v.shape[-1]
        cdt = q.dtype if q.dtype in (torch.bfloat16, torch.float16) else _mlstm_fp32_cell(q, k, v)
        lib = _lib.load()
        if not lib.sc_mlstm_supported(dtype_code(torch.empty(0, dtype=cdt)), DQ, DV):
            raise ValueError(f"mLSTM head dims (DQ={DQ}, DV={DV}) not compiled in")
        if T % 64:
            raise ValueError(f"T={T} must be a multiple of 64 (the reference pads to 64)")
        BH, nc = B * NH, T // 64
        qc, kc, vc = (x.to(cdt).contiguous().view(BH, T, -1) for x in (q, k, v))
        ig = igate.float().contiguous().view(BH, T)
        fg = fgate.float().contiguous().view(BH, T)
        c0c = None if c0 is None else c0.float().contiguous()
        n0c = None if n0 is None else n0.float().contiguous()
        m0c = None if m0 is None else m0.float().contiguous()
        dev = q.device
        h = torch.empty(BH, T, DV, dtype=cdt, device=dev)
        Cs = torch.empty(BH, nc, DV, DQ, dtype=cdt, device=dev)   # chunk-start state images [j][i]
        cT = torch.empty(B, NH, DQ, DV, dtype=torch.float32, device=dev)
        ns = torch.empty(BH, nc + 1, DQ, dtype=torch.float32, device=dev)
        ms = torch.empty(BH, nc + 1, dtype=torch.float32, device=dev)
        mrow = torch.empty(BH, T, dtype=torch.float32, device=dev)
        den = torch.empty(BH, T, dtype=torch.float32, device=dev)
        fwd_b = BH * T * (2 * DQ + 2 * DV) * qc.element_size()   # algorithmic: q k v in, h out
        with _timed("mlstm_fwd", qc, fwd_b):
            rc = lib.sc_mlstm_fwd(ptr(qc), ptr(kc), ptr(vc), dtype_code(qc), ptr(ig), ptr(fg), ptr(c0c),
                                  ptr(n0c), ptr(m0c), BH, T, DQ, DV, float(eps), ptr(h), ptr(Cs),
                                  ptr(ns), ptr(ms), ptr(cT), ptr(mrow), ptr(den), None,
                                  stream_of(qc))
        check(rc, "sc_mlstm_fwd")
        ctx.save_for_backward(qc, kc, vc, ig, fg, h, Cs, ns, ms, mrow, den)
        ctx.meta = (B, NH, T, DQ, DV, float(eps), q.dtype, k.dtype, v.dtype, c0 is not None,
                    n0 is not None)
        nT = ns[:, nc].view(B, NH, DQ).clone()
        mT = ms[:, nc].view(B, NH, 1).clone()
        ctx.mark_non_differentiable(mT)
        return h.view(B, NH, T, DV).to(q.dtype), cT, nT, mT

    @staticmethod
    def backward(ctx, dh, dcT, dnT, dmT):
        qc, kc, vc, ig, fg, h, Cs, ns, ms, mrow, den = ctx.saved_tensors
        B, NH, T, DQ, DV, eps, qdt, kdt, vdt, has_c0, has_n0 = ctx.meta
        BH, nc = B * NH, T // 64
        dev = qc.device
        if dh is None:
            dh = torch.zeros(B, NH, T, DV, dtype=qc.dtype, device=dev)
        dhc = dh.to(qc.dtype).contiguous().view(BH, T, DV)
        dcTc = None if dcT is None else dcT.float().contiguous()
        dnTc = None if dnT is None else dnT.float().contiguous()
        dCs = torch.empty(BH, DQ, DV, dtype=torch.float32, device=dev)   # d initial state
        dns = torch.empty(BH, DQ, dtype=torch.float32, device=dev)
        dq = torch.empty_like(qc)
        dk = torch.empty_like(kc)
        dv = torch.empty_like(vc)
        qdq = torch.empty(BH, T, dtype=torch.float32, device=dev)
        kdk = torch.empty(BH, T, dtype=torch.float32, device=dev)
        # algorithmic: reads q k v h dh, writes dq dk dv
        bwd_b = BH * T * (4 * DQ + 4 * DV) * qc.element_size()
        with _timed("mlstm_bwd", qc, bwd_b):
            rc = _lib.load().sc_mlstm_bwd(
                ptr(qc), ptr(kc), ptr(vc), dtype_code(qc), ptr(ig), ptr(fg), ptr(h), ptr(dhc),
                ptr(dcTc), ptr(dnTc), ptr(Cs), ptr(ns), ptr(ms), ptr(mrow), ptr(den), BH, T, DQ, DV,
                eps, ptr(dCs), ptr(dns), ptr(dq), ptr(dk), ptr(dv), ptr(qdq), ptr(kdk), None,
                stream_of(qc))
        check(rc, "sc_mlstm_bwd")
        # d igate_s = k_s.dk_s ; dF_t = q_t.dq_t - k_t.dk_t ; d fgate = sigmoid(-f) revcumsum(dF)
        dfg = torch.empty_like(kdk)
        check(_lib.load().sc_mlstm_gate_bwd(ptr(qdq), ptr(kdk), ptr(fg), BH, T, ptr(dfg), None, None,
                                            0, 0, 0, 0, 0.0, stream_of(qc)), "sc_mlstm_gate_bwd")
        shp = (B, NH, T)
        return (dq.view(B, NH, T, DQ).to(qdt), dk.view(B, NH, T, DQ).to(kdt),
                dv.view(B, NH, T, DV).to(vdt), kdk.view(shp), dfg.view(shp),
                dCs.view(B, NH, DQ, DV) if has_c0 else None,
                dns.view(B, NH, DQ) if has_n0 else None, None, None)


def _soft_cap(x, cap):
    return x if cap is None else cap * torch.tanh(x / cap)


def _soft_cap_bwd(g, x, cap):
    """d soft_cap(x) as autograd computes it in x's dtype (Mul, Tanh, Div backward)."""
    if cap is None:
        return g
    return torch.ops.aten.tanh_backward(g * cap, torch.tanh(x / cap)) / cap


class MLSTMCoreFn(torch.autograd.Function):
    """The xLSTM mLSTMLayer between its fused projection and out_proj (modeling_xlstm.py
    mLSTMLayer.forward; xlstm.mLSTMLayer): for a = [q | k | v | o | i | f] bf16 [B, T, N] (heads
    NH, per-head DQ / DV) it returns y = bf16(sigmoid(o)) * MultiHeadLayerNorm(h) [B, T, NH DV]
    with h = mLSTM(q, k, v, soft_cap(i), soft_cap(f)), and the final state (C, n, m).

    q, k, v and o are read in place from a (sc_mlstm_* layout strides, the gated norm's row
    stride): no split copies or head transposes.  The backward writes dq / dk / dv / do / di / df
    straight into ONE gradient tensor of a's shape: no concatenation of six slice gradients.
    The forward runs the same kernels and roundings as MLSTMFn + GatedHeadNormFn + the torch
    soft caps (bit-identical output and state).  The backward does not round the same way: the
    gate gradients go through the soft cap in fp32 with ONE bf16 rounding (sc_mlstm_gate_bwd),
    where the composed path and the reference's autocast chain round after each of five bf16
    ops; the gradients agree to 1e-2 relative Frobenius (measured ~1e-3,
    tests/test_gpu_xlstm_glue.py::test_mlstm_core_equals_composed_ops).
    cell_dtype: the cell's compute dtype -- bf16, or float16 as the reference configures it
    (autocast_kernel_dtype, model.py:227): q / k / v are then rounded to f16 on load inside the
    kernels (sc_mlstm_*_io), as the split path's .to(float16) rounds them, and h / dq / dk / dv
    stay bf16 in HBM."""

    @staticmethod
    def forward(ctx, a, c0, n0, m0, w_mh, NH, DQ, DV, cap, eps, eps_mh, cell_dtype=torch.bfloat16):
        require_device(a)
        ctx.set_materialize_grads(False)   # detached carried states: no zero-filled gradients
        B, T, N = a.shape
        lib = _lib.load()
        qo, ko, vo = 0, NH * DQ, 2 * NH * DQ
        oo = vo + NH * DV
        io, fo = oo + NH * DV, oo + NH * DV + NH
        BH, nc = B * NH, T // 64
        ig_raw, fg_raw = a[..., io:io + NH], a[..., fo:fo + NH]
        ig = _soft_cap(ig_raw, cap).transpose(1, 2).float().contiguous()
        fg = _soft_cap(fg_raw, cap).transpose(1, 2).float().contiguous()
        c0c = None if c0 is None else c0.float().contiguous()
        n0c = None if n0 is None else n0.float().contiguous()
        m0c = None if m0 is None else m0.float().contiguous()
        dev = a.device
        esz = a.element_size()
        base = a.data_ptr()
        lay = (ctypes.c_int64 * 7)(NH, T * N, DQ, N, T * N, DV, N)
        h = torch.empty(BH, T, DV, dtype=cell_dtype, device=dev)   # the cell's output dtype
        Cs = torch.empty(BH, nc, DV, DQ, dtype=cell_dtype, device=dev)   # state images [j][i]
        cdc = dtype_code(Cs)
        cT = torch.empty(B, NH, DQ, DV, dtype=torch.float32, device=dev)
        ns = torch.empty(BH, nc + 1, DQ, dtype=torch.float32, device=dev)
        ms = torch.empty(BH, nc + 1, dtype=torch.float32, device=dev)
        mrow = torch.empty(BH, T, dtype=torch.float32, device=dev)
        den = torch.empty(BH, T, dtype=torch.float32, device=dev)
        fwd_b = BH * T * (2 * DQ + 2 * DV) * esz   # algorithmic: q k v in, h out
        stream = stream_of(a)
        with _timed("mlstm_fwd", a, fwd_b):
            rc = lib.sc_mlstm_fwd_io(base + qo * esz, base + ko * esz, base + vo * esz, cdc,
                                     dtype_code(a), ptr(ig), ptr(fg), ptr(c0c), ptr(n0c), ptr(m0c),
                                     BH, T, DQ, DV, float(eps), ptr(h), ptr(Cs), ptr(ns), ptr(ms),
                                     ptr(cT), ptr(mrow), ptr(den), lay, stream)
        check(rc, "sc_mlstm_fwd")
        wf = w_mh.detach().float().contiguous()
        y = torch.empty(B, T, NH * DV, dtype=torch.bfloat16, device=dev)
        mean = torch.empty(B * T, NH, dtype=torch.float32, device=dev)
        rstd = torch.empty_like(mean)
        # (an f16 h is read rounded to bf16: the split path's h.to(bfloat16))
        mh_fwd = lib.sc_mhln_gate_fwd_h16 if h.dtype == torch.float16 else lib.sc_mhln_gate_fwd
        check(mh_fwd(ptr(h), base + oo * esz, N, ptr(wf), ptr(y), ptr(mean), ptr(rstd),
                     B, T, NH, DV, float(eps_mh), stream), "sc_mhln_gate_fwd")
        ctx.save_for_backward(a, ig, fg, h, Cs, ns, ms, mrow, den, wf, mean, rstd)
        ctx.meta = (NH, DQ, DV, cap, float(eps), c0 is not None, n0 is not None, w_mh.dtype)
        nT = ns[:, nc].view(B, NH, DQ).clone()
        mT = ms[:, nc].view(B, NH, 1).clone()
        ctx.mark_non_differentiable(mT)
        return y, cT, nT, mT

    @staticmethod
    def backward(ctx, dy, dcT, dnT, dmT):
        a, ig, fg, h, Cs, ns, ms, mrow, den, wf, mean, rstd = ctx.saved_tensors
        NH, DQ, DV, cap, eps, has_c0, has_n0, wdt = ctx.meta
        B, T, N = a.shape
        BH, nc = B * NH, T // 64
        qo, ko, vo = 0, NH * DQ, 2 * NH * DQ
        oo = vo + NH * DV
        io, fo = oo + NH * DV, oo + NH * DV + NH
        lib = _lib.load()
        dev = a.device
        esz = a.element_size()
        base = a.data_ptr()
        stream = stream_of(a)
        if dy is None:
            dy = torch.zeros(B, T, NH * DV, dtype=torch.bfloat16, device=dev)
        dyc = dy.to(torch.bfloat16)
        if dyc.stride(2) != 1 or dyc.stride(0) != T * dyc.stride(1) or dyc.stride(1) % 4:
            dyc = dyc.contiguous()
        da = torch.empty_like(a)
        dbase = da.data_ptr()
        dh = torch.empty(h.shape, dtype=a.dtype, device=dev)   # bf16 (f16 cell: not cast)
        part = torch.empty(lib.sc_xlstm_part_rows(B * T), NH * DV, dtype=torch.float32, device=dev)
        mh_bwd = lib.sc_mhln_gate_bwd_h16 if h.dtype == torch.float16 else lib.sc_mhln_gate_bwd
        check(mh_bwd(ptr(h), base + oo * esz, N, ptr(wf), ptr(mean), ptr(rstd),
                     ptr(dyc), dyc.stride(1), ptr(dh), dbase + oo * esz, N, ptr(part),
                     B, T, NH, DV, stream), "sc_mhln_gate_bwd")
        dcTc = None if dcT is None else dcT.float().contiguous()
        dnTc = None if dnT is None else dnT.float().contiguous()
        dCs = torch.empty(BH, DQ, DV, dtype=torch.float32, device=dev)   # d initial state
        dns = torch.empty(BH, DQ, dtype=torch.float32, device=dev)
        qdq = torch.empty(BH, T, dtype=torch.float32, device=dev)
        kdk = torch.empty(BH, T, dtype=torch.float32, device=dev)
        lay = (ctypes.c_int64 * 7)(NH, T * N, DQ, N, T * N, DV, N)
        bwd_b = BH * T * (4 * DQ + 4 * DV) * esz   # algorithmic: q k v h dh in, dq dk dv out
        with _timed("mlstm_bwd", a, bwd_b):
            rc = lib.sc_mlstm_bwd_io(
                base + qo * esz, base + ko * esz, base + vo * esz, dtype_code(Cs), dtype_code(a),
                ptr(ig), ptr(fg), ptr(h), ptr(dh), ptr(dcTc), ptr(dnTc), ptr(Cs), ptr(ns), ptr(ms), ptr(mrow),
                ptr(den), BH, T, DQ, DV, eps, ptr(dCs), ptr(dns), dbase + qo * esz,
                dbase + ko * esz, dbase + vo * esz, ptr(qdq), ptr(kdk), lay, stream)
        check(rc, "sc_mlstm_bwd")
        # gate gradients as MLSTMFn returns them, then through the soft caps (fp32, one bf16
        # rounding; _soft_cap_bwd's torch chain rounds each op) straight into da: one kernel
        check(lib.sc_mlstm_gate_bwd(ptr(qdq), ptr(kdk), ptr(fg), BH, T, None, base, dbase, NH, N,
                                    io, fo, float(cap) if cap is not None else 0.0, stream),
              "sc_mlstm_gate_bwd")
        return (da, dCs.view(B, NH, DQ, DV) if has_c0 else None,
                dns.view(B, NH, DQ) if has_n0 else None, None,
                _part_sum(part).to(wdt), None, None, None, None, None, None, None)


def mlstm_core_supported(a, NH, DQ, DV):
    """MLSTMCoreFn's preconditions: bf16 ROCm a [B, T, N] contiguous, T % 64 == 0, the head
    dims compiled in, 16-byte aligned row pieces for the strided reads."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and a.dim() == 3 and a.is_contiguous()):
        return False
    B, T, N = a.shape
    return (T % 64 == 0 and N == 2 * NH * DQ + 2 * NH * DV + 2 * NH and N % 8 == 0
            and DQ % 8 == 0 and DV % 8 == 0 and NH <= 4 and DV in (64, 128, 192, 256)
            and a.data_ptr() % 16 == 0
            and bool(_lib.load().sc_mlstm_supported(_lib.SC_BF16, DQ, DV)))


def mlstm_chunkwise(query, key, value, igate, fgate, c_initial=None, n_initial=None,
                    m_initial=None, return_last_states=False, eps=1e-6, chunk_size=64, **kwargs):
    """transformers' mlstm_chunkwise_native_autograd interface on the HIP kernels (chunk 64)."""
    if chunk_size != 64:
        raise ValueError("the HIP mLSTM kernels use chunk_size 64")
    h, c, n, m = MLSTMFn.apply(query, key, value, igate, fgate, c_initial, n_initial, m_initial, eps)
    return (h, (c, n, m)) if return_last_states else h


# ----------------------------------------------------------------------------- xLSTM glue ----
def _part_sum(part):
    """fixed-order fp32 sum of the [P, D] weight-gradient partial rows (sc_colsum)."""
    return colsum(part)


def xlstm_glue_supported(x, D):
    return x.is_cuda and x.dtype == torch.bfloat16 and D in (256, 512, 768, 1024)


class RMSNormFn(torch.autograd.Function):
    """xLSTM RMSNorm (force_float32_reductions; transformers modeling_xlstm.py RMSNorm) in one pass:
    y = bf16(bf16(x rsqrt(mean x^2 + eps)) w), the value autocast hands the next bf16 GEMM."""

    @staticmethod
    def forward(ctx, x, w, eps):
        require_device(x)
        D = x.shape[-1]
        x2 = x.reshape(-1, D)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        rows = x2.shape[0]
        wf = w.detach().float().contiguous()
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        check(_lib.load().sc_rmsnorm_fwd(ptr(x2), ptr(wf), ptr(y), ptr(rstd), rows, D, float(eps),
                                         stream_of(x2)), "sc_rmsnorm_fwd")
        ctx.save_for_backward(x2, wf, rstd)
        ctx.wdt = w.dtype
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, dy):
        x2, wf, rstd = ctx.saved_tensors
        rows, D = x2.shape
        dy2 = dy.reshape(rows, D).to(torch.bfloat16).contiguous()
        lib = _lib.load()
        dx = torch.empty_like(x2)
        part = torch.empty(lib.sc_xlstm_part_rows(rows), D, dtype=torch.float32, device=x2.device)
        check(lib.sc_rmsnorm_bwd(ptr(x2), ptr(dy2), ptr(wf), ptr(rstd), ptr(dx), ptr(part), rows, D,
                                 stream_of(x2)), "sc_rmsnorm_bwd")
        return dx.view(dy.shape), _part_sum(part).to(ctx.wdt), None


def rms_norm(x, w, eps):
    return RMSNormFn.apply(x, w, eps)


class AddRMSNormFn(torch.autograd.Function):
    """(s, n) = (x + r, RMSNorm(x + r)) in one pass: the xLSTM block's residual add folded into
    the RMSNorm that reads its result (sc_rmsnorm_add_fwd).  The backward folds the residual
    branch's gradient ds into the norm's dx (sc_rmsnorm_add_bwd), so neither the forward add nor
    autograd's gradient accumulation is a kernel of its own; bf16 roundings as the torch chain."""

    @staticmethod
    def forward(ctx, x, r, w, eps):
        require_device(x, r)
        D = x.shape[-1]
        x2 = x.reshape(-1, D)
        r2 = r.reshape(-1, D)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        if not r2.is_contiguous():
            r2 = r2.contiguous()
        rows = x2.shape[0]
        wf = w.detach().float().contiguous()
        s = torch.empty_like(x2)
        y = torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        check(_lib.load().sc_rmsnorm_add_fwd(ptr(x2), ptr(r2), ptr(s), ptr(wf), ptr(y), ptr(rstd),
                                             rows, D, float(eps), stream_of(x2)),
              "sc_rmsnorm_add_fwd")
        ctx.save_for_backward(s, wf, rstd)
        ctx.wdt = w.dtype
        return s.view(x.shape), y.view(x.shape)

    @staticmethod
    def backward(ctx, ds, dy):
        s, wf, rstd = ctx.saved_tensors
        rows, D = s.shape
        lib = _lib.load()
        if dy is None:   # the normalised output unused: the add's own gradient only
            return ds, ds, None, None
        dy2 = dy.reshape(rows, D).to(torch.bfloat16).contiguous()
        dx = torch.empty_like(s)
        part = torch.empty(lib.sc_xlstm_part_rows(rows), D, dtype=torch.float32, device=s.device)
        if ds is None:
            check(lib.sc_rmsnorm_bwd(ptr(s), ptr(dy2), ptr(wf), ptr(rstd), ptr(dx), ptr(part), rows,
                                     D, stream_of(s)), "sc_rmsnorm_bwd")
        else:
            ds2 = ds.reshape(rows, D).to(torch.bfloat16).contiguous()
            check(lib.sc_rmsnorm_add_bwd(ptr(s), ptr(dy2), ptr(ds2), ptr(wf), ptr(rstd), ptr(dx),
                                         ptr(part), rows, D, stream_of(s)), "sc_rmsnorm_add_bwd")
        dx = dx.view(dy.shape)
        return dx, dx, _part_sum(part).to(ctx.wdt), None


def add_rms_norm(x, r, w, eps):
    """(x + r, RMSNorm(x + r)) through AddRMSNormFn (bf16 ROCm tensors, xlstm_glue_supported)."""
    return AddRMSNormFn.apply(x, r, w, eps)


class GatedHeadNormFn(torch.autograd.Function):
    """bf16(sigmoid(o)) * MultiHeadLayerNorm(h) of the mLSTM layer (modeling_xlstm.py mLSTMLayer:
    out_proj(sigmoid(o) * multihead_norm(h))) in one pass: h [B,NH,T,DH] the cell output in the
    cell's own layout, o [B,T,NH*DH] a row-strided view of the fused projection; out bf16
    [B,T,NH*DH].  Backward: dh [B,NH,T,DH], do [B,T,NH*DH], d weight."""

    @staticmethod
    def forward(ctx, h, o, w, eps):
        require_device(h, o)
        B, NH, T, DH = h.shape
        h = h.contiguous()
        if o.stride(2) != 1 or o.stride(0) != T * o.stride(1) or o.stride(1) % 4:
            o = o.contiguous()
        wf = w.detach().float().contiguous()
        out = torch.empty(B, T, NH * DH, dtype=torch.bfloat16, device=h.device)
        mean = torch.empty(B * T, NH, dtype=torch.float32, device=h.device)
        rstd = torch.empty_like(mean)
        check(_lib.load().sc_mhln_gate_fwd(ptr(h), ptr(o), o.stride(1), ptr(wf), ptr(out), ptr(mean),
                                           ptr(rstd), B, T, NH, DH, float(eps), stream_of(h)),
              "sc_mhln_gate_fwd")
        ctx.save_for_backward(h, o, wf, mean, rstd)
        ctx.wdt = w.dtype
        return out

    @staticmethod
    def backward(ctx, dout):
        h, o, wf, mean, rstd = ctx.saved_tensors
        B, NH, T, DH = h.shape
        dy = dout.to(torch.bfloat16)
        if dy.stride(2) != 1 or dy.stride(0) != T * dy.stride(1) or dy.stride(1) % 4:
            dy = dy.contiguous()
        lib = _lib.load()
        dh = torch.empty_like(h)
        do = torch.empty(B, T, NH * DH, dtype=torch.bfloat16, device=h.device)
        part = torch.empty(lib.sc_xlstm_part_rows(B * T), NH * DH, dtype=torch.float32,
                           device=h.device)
        check(lib.sc_mhln_gate_bwd(ptr(h), ptr(o), o.stride(1), ptr(wf), ptr(mean), ptr(rstd), ptr(dy),
                                   dy.stride(1), ptr(dh), ptr(do), do.stride(1), ptr(part), B, T, NH,
                                   DH, stream_of(h)), "sc_mhln_gate_bwd")
        return dh, do, _part_sum(part).to(ctx.wdt), None


def gated_head_norm(h, o, w, eps):
    return GatedHeadNormFn.apply(h, o, w, eps)


def gated_head_norm_supported(h):
    return (h.is_cuda and h.dtype == torch.bfloat16 and h.dim() == 4 and h.shape[1] <= 4
            and h.shape[3] in (64, 128, 192, 256))


class SwiGLUFn(torch.autograd.Function):
    """bf16(silu(g)) * u for a = [g | u] (the fused up-projection of the xLSTM FFN); the
    backward returns ONE [dg | du] tensor (no concatenation of two slice gradients)."""

    @staticmethod
    def forward(ctx, a):
        require_device(a)
        F2 = a.shape[-1]
        a2 = a.reshape(-1, F2).contiguous()
        y = torch.empty(a2.shape[0], F2 // 2, dtype=torch.bfloat16, device=a.device)
        check(_lib.load().sc_swiglu_fwd(ptr(a2), ptr(y), a2.shape[0], F2 // 2, stream_of(a2)),
              "sc_swiglu_fwd")
        ctx.save_for_backward(a2)
        return y.view(*a.shape[:-1], F2 // 2)

    @staticmethod
    def backward(ctx, dy):
        (a2,) = ctx.saved_tensors
        rows, F2 = a2.shape
        dy2 = dy.reshape(rows, F2 // 2).to(torch.bfloat16).contiguous()
        da = torch.empty_like(a2)
        check(_lib.load().sc_swiglu_bwd(ptr(a2), ptr(dy2), ptr(da), rows, F2 // 2, stream_of(a2)),
              "sc_swiglu_bwd")
        return da.view(*dy.shape[:-1], F2)


def swiglu(a):
    return SwiGLUFn.apply(a)


_MM_DTYPE = [True]


def _mm_f32(a, b):
    """a @ b with fp32 output for bf16 operands (aten::mm.dtype: fp32 accumulate, no rounding
    of the product to bf16), or in fp32 when that overload is unavailable."""
    if _MM_DTYPE[0]:
        try:
            return torch.mm(a, b, out_dtype=torch.float32)
        except (RuntimeError, TypeError, NotImplementedError):
            _MM_DTYPE[0] = False
    return a.float() @ b.float()


class AutocastLinearFn(torch.autograd.Function):
    """y = x W^T (+ b) in the autocast dtype (what nn.Linear does under bf16 autocast) with a
    backward that takes the weight gradient from the MFMA split-L kernel when the shape fits
    (dW = dY^T X reduces over the B*T rows, hipBLASLt's weakest case): the xLSTM blocks' linears.
    The input gradient stays a library GEMM (NN form, TunableOp table)."""

    @staticmethod
    def forward(ctx, x, w, b, cdt, bias_from=0):
        xc = x.to(cdt)
        wc = w.to(cdt)
        with _timed("xlstm_gemm", xc, 0, 2 * xc.numel() * wc.shape[0]):
            y = torch.nn.functional.linear(xc, wc, None if b is None else b.to(cdt))
        ctx.save_for_backward(xc, wc)
        ctx.meta = (x.dtype, w.dtype, None if b is None else b.dtype)
        ctx.bias_from = bias_from
        return y

    @staticmethod
    def backward(ctx, dy):
        dx, dw, db = _linear_grads(ctx, dy, *ctx.needs_input_grad[:3])
        return dx, dw, db, None, None


def _linear_grads(ctx, dy, need_x, need_w, need_b):
    """(dx, dW, db) of AutocastLinearFn / FusedLinearFn from the saved (xc, wc), ctx.meta and
    ctx.bias_from."""
    xc, wc = ctx.saved_tensors
    xdt, wdt, bdt = ctx.meta
    N, K = wc.shape
    dy2 = dy.reshape(-1, N).to(wc.dtype)
    x2 = xc.reshape(-1, K)
    dx = dw = db = None
    gemm_flops = 2 * dy2.shape[0] * N * K
    if need_x:
        with _timed("xlstm_gemm", dy2, 0, gemm_flops):
            dx = dy2 @ wc
        dx = dx.view(*dy.shape[:-1], K).to(xdt)
    if need_w:
        tw = _timed("xlstm_gemm", dy2, 0, gemm_flops)
        tw.__enter__()
        dw = None
        if dy2.is_cuda and dy2.dtype == torch.bfloat16:
            dyc, xcc = dy2.contiguous(), x2.contiguous()
            dw = wgrad_mfma(dyc, xcc)
            n0 = N - N % 256
            if dw is None and 256 <= n0 < N:
                # e.g. the xLSTM q|k|v|o|i|f projection (N = 2312 at C4): the first N0 rows
                # of dW on the MFMA kernel (dy's row stride 2312 is a multiple of 8), the
                # gate rows that remain as a small library GEMM
                head = wgrad_mfma(dyc[:, :n0], xcc)
                if head is not None:
                    # the tail rows from the MFMA kernel too, over the last 256-row window
                    # (a 16-byte aligned view when N % 8 == 0; its first rows repeat the
                    # head's): an M = 8, K = 48000 library GEMM took 130 us at C4, the
                    # window ~30 us
                    win = wgrad_mfma(dyc[:, N - 256:], xcc)
                    tail = win[256 - (N - n0):] if win is not None else \
                        _mm_f32(dyc[:, n0:].t(), xcc)
                    dw = torch.cat([head, tail])
        dw = (dw if dw is not None else (dy2.t() @ x2).float())
        tw.__exit__()
        dw = dw.to(wdt)
    if bdt is not None and need_b:
        f = ctx.bias_from
        if f and f < N and (f * dy2.element_size()) % 16 == 0:
            # bias entries before `f` are constant zero pieces (the xLSTM projection's
            # q|k|v|o part): only the gate columns are summed over the B*T rows
            db = torch.cat([torch.zeros(f, dtype=torch.float32, device=dy2.device),
                            colsum(dy2[:, f:])]).to(bdt)
        else:
            db = colsum(dy2).to(bdt)
    return dx, dw, db


class FusedLinearFn(torch.autograd.Function):
    """AutocastLinearFn over the row-concatenation of several fp32 weights (the xLSTM fused
    projections) without materialising the fp32 concatenation: the bf16 image [sum rows, K] is
    written by ONE sc_weight_images launch (cast and concatenation together), and the weight
    gradient is split back into one gradient per weight.  Same roundings as cat -> cast."""

    @staticmethod
    def forward(ctx, x, b, cdt, bias_from, *ws):
        rows = [w.shape[0] for w in ws]
        K = ws[0].shape[1]
        wc = torch.empty(sum(rows), K, dtype=cdt, device=x.device)
        jobs, off = [], 0
        for w, r in zip(ws, rows):
            jobs.append(_lib.ImageJob(w.data_ptr(), wc[off].data_ptr(), None, r, K, K, w.stride(0), 0))
            off += r
        _image_jobs(jobs, list(ws))
        xc = x.to(cdt)
        with _timed("xlstm_gemm", xc, 0, 2 * xc.numel() * wc.shape[0]):
            y = torch.nn.functional.linear(xc, wc, None if b is None else b.to(cdt))
        ctx.save_for_backward(xc, wc)
        ctx.meta = (x.dtype, ws[0].dtype, None if b is None else b.dtype)
        ctx.bias_from = bias_from
        ctx.rows = rows
        return y

    @staticmethod
    def backward(ctx, dy):
        need = ctx.needs_input_grad
        dx, dw, db = _linear_grads(ctx, dy, need[0], any(need[4:]), need[1])
        dws = dw.split(ctx.rows) if dw is not None else [None] * len(ctx.rows)
        return (dx, db, None, None) + tuple(dws)


def fused_linear_ok(x, ws):
    """FusedLinearFn's preconditions: bf16 autocast on a ROCm device, fp32 weights with unit
    column stride and one common K."""
    return (x.is_cuda and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and all(w.is_cuda and w.dtype == torch.float32 and w.dim() == 2 and w.stride(1) == 1
                    and w.shape[1] == ws[0].shape[1] for w in ws))


def fused_linear(x, ws, b=None, bias_from=0):
    """nn.Linear under bf16 autocast with weight = torch.cat(ws) (FusedLinearFn)."""
    with torch.autocast("cuda", enabled=False):
        return FusedLinearFn.apply(x, b, torch.bfloat16, int(bias_from), *ws)


def autocast_linear(x, w, b=None, bias_from=0):
    """nn.Linear semantics under autocast (bf16 compute when enabled) through AutocastLinearFn.
    bias_from: b[:bias_from] is a constant (its gradient is not summed; the returned gradient
    there is 0)."""
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        cdt = torch.get_autocast_dtype("cuda")
    else:
        cdt = torch.promote_types(x.dtype, w.dtype)
    with torch.autocast("cuda", enabled=False):
        return AutocastLinearFn.apply(x, w, b, cdt, int(bias_from))
