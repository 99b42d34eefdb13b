"""ctypes binding of libstatecatcher_hip.so (C ABI: include/statecatcher.h).

The product path has no CPU fallback: every op raises if the library is missing, if a tensor is
not on a ROCm device, or if a call returns a non-zero status.
"""
import ctypes
import os

import torch  # noqa: F401  (loads torch's HIP runtime first: our .so binds to the same SONAME)

LIB_NAME = "libstatecatcher_hip.so"
# SC_LIB_PATH: load another build of the same ABI (ablation builds under tools/); default in-tree
LIB_PATH = os.environ.get("SC_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                         LIB_NAME)

SC_F32, SC_BF16, SC_F16 = 0, 1, 2
_DTYPE = {torch.float32: SC_F32, torch.bfloat16: SC_BF16, torch.float16: SC_F16}

_c = ctypes
_i32, _i64, _vp, _fp = _c.c_int, _c.c_int64, _c.c_void_p, _c.c_void_p
ABI_VERSION = 14  # include/statecatcher.h; bumped on any signature change

_SIGS = {
    "sc_abi_version": (_i32, []),
    "sc_gemm_wgrad_splits": (_i32, [_i32, _i32, _i32]),
    "sc_gemm_wgrad_bf16": (_i32, [_vp, _i64, _vp, _i64, _fp, _i32, _i32, _i32, _i32, _vp]),
    "sc_gemm_tn_bf16": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _i32, _vp]),
    "sc_gemm_tn_ln_bf16": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _i32, _i32, _i32, _fp, _vp,
                                 _c.c_float, _vp]),
    "sc_last_error": (_c.c_char_p, []),
    "sc_lucy_scan_chunk": (_i32, []),
    "sc_lucy_scan_ckpt_numel": (_i64, [_i32, _i32, _i32]),
    "sc_lucy_scan_fwd": (_i32, [_vp, _i32, _fp, _fp, _fp, _vp, _fp, _fp, _i32, _i32, _i32,
                               _i64, _i64, _i64, _i64, _i64, _i64, _fp, _vp]),
    "sc_lucy_scan_fwd_split": (_i32, [_vp, _i32, _fp, _fp, _fp, _vp, _vp, _vp, _fp, _fp, _i32, _i32,
                                     _i32, _i64, _i64, _i64, _i64, _i64, _i64, _fp, _vp]),
    "sc_lucy_scan_bwd": (_i32, [_vp, _i32, _fp, _fp, _vp, _fp, _vp, _fp, _fp, _fp, _i32, _i32, _i32,
                               _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                               _vp]),
    "sc_lucy_scan_fwd_ln": (_i32, [_vp, _i32, _fp, _fp, _fp, _vp, _vp, _vp, _fp, _fp, _i32, _i32,
                                  _i32, _i64, _i64, _i64, _i64, _i64, _i64, _fp, _fp, _fp, _fp, _fp,
                                  _c.c_float, _vp]),
    "sc_lucy_scan_bwd_ln": (_i32, [_vp, _i32, _fp, _fp, _vp, _fp, _vp, _fp, _fp, _fp, _i32, _i32,
                                  _i32, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64, _i64,
                                  _fp, _fp, _vp]),
    "sc_ln_fold_prep": (_i32, [_vp, _i32, _vp]),
    "sc_ln_fold_bwd": (_i32, [_vp, _vp, _i32, _fp, _vp, _i64, _i32, _vp]),
    "sc_ln_fold_wgrad_workspace_numel": (_i64, [_i32, _i32]),
    "sc_ln_fold_wgrad": (_i32, [_fp, _fp, _i64, _fp, _fp, _fp, _i32, _i32, _fp, _fp, _fp, _vp]),
    "sc_decay_scan_fwd": (_i32, [_vp, _vp, _vp, _i32, _fp, _i32, _i32, _i32, _i64, _i64, _i64, _vp]),
    "sc_decay_scan_bwd": (_i32, [_vp, _vp, _vp, _vp, _vp, _i32, _fp, _fp, _i32, _i32, _i32,
                                _i64, _i64, _i64, _vp]),
    "sc_layernorm_supported": (_i32, [_i32, _i32]),
    "sc_layernorm_fwd": (_i32, [_vp, _i32, _fp, _fp, _vp, _fp, _fp, _i64, _i32, _c.c_float, _vp]),
    "sc_layernorm_bwd_workspace_numel": (_i64, [_i64, _i32]),
    "sc_layernorm_bwd": (_i32, [_vp, _vp, _i32, _fp, _fp, _fp, _vp, _fp, _fp, _i64, _i32, _vp]),
    "sc_ctc_workspace_bytes": (_c.c_size_t, [_i32, _i32, _i32]),
    "sc_ctc_fwd": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i64, _i32, _vp, _vp,
                         _i32, _fp, _vp, _c.c_size_t, _vp]),
    "sc_ctc_bwd": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i64, _i32, _vp, _vp,
                         _i32, _fp, _fp, _vp, _i32, _vp, _c.c_size_t, _vp]),
    "sc_ctc_fwd_ex": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i64, _i32, _vp,
                            _vp, _i32, _fp, _i64, _i64, _fp, _vp, _c.c_size_t, _vp]),
    "sc_ctc_bwd_ex": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i64, _i32, _vp,
                            _vp, _i32, _fp, _i64, _i64, _fp, _fp, _vp, _i32, _vp, _c.c_size_t,
                            _vp]),
    "sc_ctc_split_rows": (_i32, [_fp, _i64, _fp, _i32, _i32, _vp, _i64, _i32, _i32, _vp, _fp,
                                 _i32, _vp]),
    "sc_ctc_greedy_decode": (_i32, [_vp, _i32, _i32, _i32, _i32, _i64, _i64, _vp, _i32, _vp, _vp, _vp]),
    "sc_colsum_workspace_bytes": (_c.c_size_t, [_i64, _i64]),
    "sc_colsum": (_i32, [_vp, _i32, _i64, _i64, _i64, _i64, _i64, _fp, _vp, _c.c_size_t, _vp]),
    "sc_fbank_frames": (_i64, [_i64]),
    "sc_fbank_workspace_bytes": (_c.c_size_t, []),
    "sc_fbank": (_i32, [_vp, _i32, _i64, _i64, _i32, _c.c_float, _fp, _vp, _c.c_size_t, _vp]),
    "sc_ctc_mean": (_i32, [_fp, _vp, _i32, _fp, _fp, _vp]),
    "sc_ctc_greedy_step": (_i32, [_vp, _i32, _i32, _i32, _i64, _fp, _i32, _vp, _vp, _i64, _vp]),
    "sc_lucy_step_supported": (_i32, [_i32, _i32]),
    "sc_lucy_step_ln": (_i32, [_vp, _i32, _fp, _fp, _c.c_float, _vp, _i32, _i32, _vp]),
    "sc_lucy_step_cell": (_i32, [_i32, _vp, _i32, _i64, _vp, _vp, _fp, _fp, _fp, _fp, _c.c_float,
                                 _fp, _fp, _vp, _fp, _i32, _i32, _vp]),
    "sc_lucy_frame_gemm": (_i32, [_i32, _fp, _i64, _i32, _fp, _fp, _vp, _i32, _c.c_float, _vp, _i32,
                                  _i64, _fp, _i32, _i32, _fp, _i64, _vp, _fp, _vp, _fp, _fp, _vp]),
    "sc_lucy_frame_cellb": (_i32, [_fp, _vp, _i32, _fp, _vp, _i32, _fp, _fp, _fp, _fp, _c.c_float,
                                   _fp, _fp, _i64, _fp, _i32, _i32, _vp]),
    "sc_lucy_frame_gemm_multi": (_i32, [_i32, _i32, _c.c_float, _vp, _i32, _vp]),
    "sc_lucy_frame_cellb_multi": (_i32, [_c.c_float, _vp, _i32, _vp]),
    "sc_ctc_greedy_frames": (_i32, [_vp, _i32, _i32, _i32, _i32, _i64, _i64, _fp, _i64, _i32, _vp,
                                    _vp, _i64, _i64, _vp]),
    "sc_mlstm_supported": (_i32, [_i32, _i32, _i32]),
    "sc_mlstm_chunk_state_numel": (_i64, [_i32, _i32, _i32, _i32]),
    "sc_mlstm_fwd": (_i32, [_vp, _vp, _vp, _i32, _fp, _fp, _fp, _fp, _fp, _i32, _i32, _i32, _i32,
                           _c.c_float, _vp, _vp, _fp, _fp, _fp, _fp, _fp, _vp, _vp]),
    "sc_mlstm_bwd": (_i32, [_vp, _vp, _vp, _i32, _fp, _fp, _vp, _vp, _fp, _fp, _vp, _fp, _fp, _fp,
                           _fp, _i32, _i32, _i32, _i32, _c.c_float, _fp, _fp, _vp, _vp, _vp, _fp,
                           _fp, _vp, _vp]),
    "sc_mlstm_fwd_io": (_i32, [_vp, _vp, _vp, _i32, _i32, _fp, _fp, _fp, _fp, _fp, _i32, _i32, _i32,
                              _i32, _c.c_float, _vp, _vp, _fp, _fp, _fp, _fp, _fp, _vp, _vp]),
    "sc_mlstm_bwd_io": (_i32, [_vp, _vp, _vp, _i32, _i32, _fp, _fp, _vp, _vp, _fp, _fp, _vp, _fp, _fp,
                              _fp, _fp, _i32, _i32, _i32, _i32, _c.c_float, _fp, _fp, _vp, _vp, _vp,
                              _fp, _fp, _vp, _vp]),
    "sc_mlstm_gate_bwd": (_i32, [_fp, _fp, _fp, _i32, _i32, _fp, _vp, _vp, _i32, _i64, _i32, _i32,
                                _c.c_float, _vp]),
    "sc_xlstm_part_rows": (_i32, [_i64]),
    "sc_rmsnorm_fwd": (_i32, [_vp, _fp, _vp, _fp, _i64, _i32, _c.c_float, _vp]),
    "sc_rmsnorm_bwd": (_i32, [_vp, _vp, _fp, _fp, _vp, _fp, _i64, _i32, _vp]),
    "sc_rmsnorm_add_fwd": (_i32, [_vp, _vp, _vp, _fp, _vp, _fp, _i64, _i32, _c.c_float, _vp]),
    "sc_rmsnorm_add_bwd": (_i32, [_vp, _vp, _vp, _fp, _fp, _vp, _fp, _i64, _i32, _vp]),
    "sc_mhln_gate_fwd": (_i32, [_vp, _vp, _i64, _fp, _vp, _fp, _fp, _i32, _i32, _i32, _i32,
                                _c.c_float, _vp]),
    "sc_mhln_gate_bwd": (_i32, [_vp, _vp, _i64, _fp, _fp, _fp, _vp, _i64, _vp, _vp, _i64, _fp,
                                _i32, _i32, _i32, _i32, _vp]),
    "sc_mhln_gate_fwd_h16": (_i32, [_vp, _vp, _i64, _fp, _vp, _fp, _fp, _i32, _i32, _i32, _i32,
                                _c.c_float, _vp]),
    "sc_mhln_gate_bwd_h16": (_i32, [_vp, _vp, _i64, _fp, _fp, _fp, _vp, _i64, _vp, _vp, _i64, _fp,
                                _i32, _i32, _i32, _i32, _vp]),
    "sc_swiglu_fwd": (_i32, [_vp, _vp, _i64, _i32, _vp]),
    "sc_swiglu_bwd": (_i32, [_vp, _vp, _vp, _i64, _i32, _vp]),
    "sc_adam_parts": (_i64, [_vp, _i32]),
    "sc_adam_sumsq": (_i32, [_vp, _i32, _fp, _vp]),
    "sc_adam_step": (_i32, [_vp, _i32, _fp, _i64, _c.c_double, _c.c_double, _c.c_double,
                           _c.c_double, _c.c_double, _c.c_double, _i32, _c.c_double, _c.c_double,
                           _fp, _vp]),
    "sc_weight_images": (_i32, [_vp, _i32, _vp]),
    "sc_rnnt_workspace_bytes": (_c.c_size_t, [_i32, _i32, _i32]),
    "sc_rnnt_joint_geometry": (_i32, [_i32, _i32, _i32, _i32, _vp, _vp, _vp]),
    "sc_rnnt_joint_fwd": (_i32, [_fp, _fp, _vp, _fp, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp,
                                 _vp, _i32, _fp, _vp, _c.c_size_t, _vp]),
    "sc_rnnt_joint_bwd": (_i32, [_fp, _fp, _vp, _fp, _i32, _i32, _i32, _i32, _i32, _vp, _i64, _vp,
                                 _vp, _i32, _fp, _fp, _fp, _fp, _fp, _vp, _c.c_size_t, _vp]),
    "sc_rnnt_fwd": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _i64, _vp, _vp, _i64,
                          _vp, _vp, _i32, _fp, _vp, _c.c_size_t, _vp]),
    "sc_rnnt_bwd": (_i32, [_vp, _i32, _i32, _i32, _i32, _i32, _i32, _i64, _i64, _i64, _vp, _vp, _i64,
                          _vp, _vp, _i32, _fp, _vp, _i32, _vp, _c.c_size_t, _vp]),
}
EXPORTED = tuple(_SIGS)


class AdamTensor(ctypes.Structure):
    """sc_adam_tensor (include/statecatcher.h)."""
    _fields_ = [("p", _vp), ("g", _vp), ("m", _vp), ("v", _vp), ("n", _i64)]


class ImageJob(ctypes.Structure):
    """sc_image_job (include/statecatcher.h)."""
    _fields_ = [("src", _vp), ("dst", _vp), ("dst_t", _vp), ("rows", _i64), ("cols", _i64),
                ("cols_pad", _i64), ("ld_src", _i64), ("block_d", _i64), ("col_scale", _vp),
                ("row_shift", _vp)]


class LnFoldJob(ctypes.Structure):
    """sc_ln_fold_job (include/statecatcher.h)."""
    _fields_ = [("w", _vp), ("gamma", _vp), ("beta", _vp), ("bias", _vp), ("shift", _vp),
                ("bias_out", _vp), ("rowsum", _vp), ("ld", _i64), ("rows", _i64), ("D", _i64)]


class FrameGemmJob(ctypes.Structure):
    """sc_frame_gemm_job (include/statecatcher.h)."""
    _fields_ = [("x", _vp), ("ldx", _i64), ("K", _i32), ("ln_w", _vp), ("ln_b", _vp),
                ("st_in", _vp), ("nst_in", _i32), ("w", _vp), ("ldw", _i64), ("bias", _vp),
                ("B", _i32), ("N", _i32), ("y", _vp), ("ldy", _i64), ("st_out", _vp), ("z", _vp),
                ("st_z", _vp), ("s", _vp), ("mask", _vp)]


class FrameCellJob(ctypes.Structure):
    """sc_frame_cell_job (include/statecatcher.h)."""
    _fields_ = [("z", _vp), ("st_z", _vp), ("nst_z", _i32), ("hp", _vp), ("st_h", _vp),
                ("nst_h", _i32), ("lnz_w", _vp), ("lnz_b", _vp), ("lnh_w", _vp), ("lnh_b", _vp),
                ("h", _vp), ("out", _vp), ("ldo", _i64), ("mask", _vp), ("B", _i32), ("D", _i32)]


_LIB = None


def load():
    """Load (once) and return the ctypes handle.  Raises RuntimeError if it is not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"statecatcher HIP library not built: {LIB_PATH} missing "
                "(run `python -c 'import __graft_entry__ as g; g.build()'` or "
                "`make -C statecatcher_amd/csrc`)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.sc_abi_version() != ABI_VERSION:
            raise RuntimeError("statecatcher ABI version mismatch")
        _LIB = lib
    return _LIB


def check(rc, what):
    if rc != 0:
        msg = load().sc_last_error().decode(errors="replace")
        if rc < 0:
            raise ValueError(f"{what}: {msg}")
        raise RuntimeError(f"{what}: HIP error {rc}: {msg}")


def dtype_code(t):
    try:
        return _DTYPE[t.dtype]
    except KeyError:
        raise TypeError(f"unsupported dtype {t.dtype}; expected float32, bfloat16 or float16") from None


def require_device(*tensors):
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise RuntimeError(
                "statecatcher ops run only on a ROCm GPU (HIP); got a tensor on "
                f"{t.device}. There is no CPU fallback.")


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None
