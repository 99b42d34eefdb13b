"""CPU checks of the C ABI: the library loads here (no GPU) and exports every symbol that
include/statecatcher.h declares; argument validation returns SC_EINVAL without touching a GPU."""
import ctypes
import os
import re

import pytest

from tests.conftest import ROOT

HEADER = os.path.join(ROOT, "include", "statecatcher.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(sc_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def lib():
    from statecatcher_amd import _lib
    return _lib.load()


def test_library_exports_every_header_symbol(lib):
    names = header_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n


def test_binding_covers_header(lib):
    from statecatcher_amd import _lib
    assert sorted(_lib.EXPORTED) == header_functions()


def test_abi_version_and_sizes(lib):
    assert lib.sc_abi_version() == 14
    assert lib.sc_lucy_scan_chunk() == 64
    assert lib.sc_lucy_scan_ckpt_numel(32, 1500, 512) == 32 * 24 * 2 * 512
    assert lib.sc_lucy_scan_ckpt_numel(2, 64, 3) == 2 * 1 * 2 * 3
    assert lib.sc_lucy_scan_ckpt_numel(2, 65, 3) == 2 * 2 * 2 * 3
    assert lib.sc_ctc_workspace_bytes(32, 1500, 150) >= 32 * 1500 * (2 * 301 + 1) * 4


def test_invalid_arguments_rejected_without_gpu(lib):
    null = ctypes.c_void_p()
    rc = lib.sc_lucy_scan_fwd(null, 7, null, null, null, null, null, null, 1, 1, 1, 1, 1, 1, 64, 1, 1, null, null)
    assert rc == -1
    assert b"dtype" in lib.sc_last_error()
    rc = lib.sc_lucy_scan_fwd(null, 0, null, null, null, null, null, null, -1, 1, 1, 1, 1, 1, 64, 1, 1, null, null)
    assert rc == -1
    rc = lib.sc_decay_scan_fwd(null, null, null, 0, null, 1, 1, 1, 1, 1, 2, null)
    assert rc == -1 and b"stride_d" in lib.sc_last_error()
    rc = lib.sc_ctc_fwd(null, 0, 1, 1, 1, 4, 4, 4, null, 0, 1008, null, null, 0, null, null, 0, null)
    assert rc == -1 and b"exceeds" in lib.sc_last_error()
    rc = lib.sc_ctc_fwd(null, 0, 1, 1, 1, 4, 4, 4, null, 0, 1, null, null, 9, null, null, 0, null)
    assert rc == -1 and b"blank" in lib.sc_last_error()
    # empty problems are no-ops
    assert lib.sc_lucy_scan_fwd(null, 0, null, null, null, null, null, null, 0, 5, 5, 1, 1, 1, 64, 1, 1, null, null) == 0
    assert lib.sc_ctc_greedy_decode(null, 0, 0, 5, 5, 1, 1, null, 0, null, null, null) == 0


def test_round4_entry_points_reject_bad_arguments_without_gpu(lib):
    """The split-precision scan and the streaming frame kernels validate before launching."""
    null = ctypes.c_void_p()
    # split planes need a 16-bit out
    rc = lib.sc_lucy_scan_fwd_split(null, 0, null, null, null, null, null, null, null, null, 1, 1, 64,
                                    1, 1, 1, 64, 1, 1, null, null)
    assert rc == -1 and b"16-bit" in lib.sc_last_error()
    # frame GEMM: bad epilogue, bad weight dtype, cell shape
    rc = lib.sc_lucy_frame_gemm(9, null, 4, 4, null, null, null, 0, ctypes.c_float(1e-5), null, 0, 8,
                                null, 1, 64, null, 4, null, null, null, null, null, null)
    assert rc == -1 and b"epilogue" in lib.sc_last_error()
    rc = lib.sc_lucy_frame_gemm(0, null, 4, 4, null, null, null, 0, ctypes.c_float(1e-5), null, 2, 8,
                                null, 1, 64, null, 4, null, null, null, null, null, null)
    assert rc == -1 and b"fp32 or bf16" in lib.sc_last_error()
    assert lib.sc_lucy_frame_gemm(0, null, 4, 4, null, null, null, 0, ctypes.c_float(1e-5), null, 0,
                                  8, null, 0, 64, null, 4, null, null, null, null, null, null) == 0
    rc = lib.sc_lucy_frame_cellb(null, null, 0, null, null, 0, null, null, null, null,
                                 ctypes.c_float(1e-5), null, null, 4, null, 1, 16, null)
    assert rc == -1 and b"null" in lib.sc_last_error()


def test_frame_multi_entry_points_reject_bad_arguments_without_gpu(lib):
    """sc_lucy_frame_gemm_multi / _cellb_multi / sc_ctc_greedy_frames (ABI v13) validate every job
    before launching; empty calls are no-ops."""
    from statecatcher_amd._lib import FrameCellJob, FrameGemmJob
    null = ctypes.c_void_p()
    assert lib.sc_lucy_frame_gemm_multi(0, 0, ctypes.c_float(1e-5), null, 0, null) == 0
    rc = lib.sc_lucy_frame_gemm_multi(0, 0, ctypes.c_float(1e-5), null, 9, null)
    assert rc == -1 and b"jobs per call" in lib.sc_last_error()
    jobs = (FrameGemmJob * 2)()
    jobs[0].B, jobs[0].K, jobs[0].N = 1, 4, 64     # job 0: null pointers
    rc = lib.sc_lucy_frame_gemm_multi(0, 0, ctypes.c_float(1e-5), jobs, 2, null)
    assert rc == -1 and b"null" in lib.sc_last_error()
    rc = lib.sc_lucy_frame_gemm_multi(7, 0, ctypes.c_float(1e-5), jobs, 2, null)
    assert rc == -1 and b"epilogue" in lib.sc_last_error()
    cj = (FrameCellJob * 1)()
    cj[0].B, cj[0].D = 1, 16
    rc = lib.sc_lucy_frame_cellb_multi(ctypes.c_float(1e-5), cj, 1, null)
    assert rc == -1 and b"null" in lib.sc_last_error()
    assert lib.sc_ctc_greedy_frames(null, 0, 0, 4, 8, 32, 8, null, 4, 0, null, null, 4, 1, null) == 0
    rc = lib.sc_ctc_greedy_frames(null, 5, 2, 4, 8, 32, 8, null, 4, 0, null, null, 4, 1, null)
    assert rc == -1 and b"dtype" in lib.sc_last_error()


def test_ctc_side_array_entry_points_reject_bad_arguments_without_gpu(lib):
    """sc_ctc_fwd_ex / sc_ctc_bwd_ex / sc_ctc_split_rows (ABI v10-11) validate before launching:
    emission logits need is_logits and rows of max_target_len + 1; split rows need aligned rows
    and a blank inside V; empty batches are no-ops."""
    null = ctypes.c_void_p()
    fake = ctypes.c_void_p(0x1000)   # never dereferenced: validation fails first
    ws = lib.sc_ctc_workspace_bytes(2, 10, 3)
    # is_logits = 0 with emission logits
    rc = lib.sc_ctc_fwd_ex(fake, 0, 0, 2, 10, 8, 80, 8, fake, 3, 3, fake, fake, 0, fake, 40, 4,
                           fake, fake, ws, null)
    assert rc == -1 and b"is_logits" in lib.sc_last_error()
    # rows shorter than max_target_len + 1
    rc = lib.sc_ctc_fwd_ex(fake, 0, 1, 2, 10, 8, 80, 8, fake, 3, 3, fake, fake, 0, fake, 40, 3,
                           fake, fake, ws, null)
    assert rc == -1 and b"max_target_len + 1" in lib.sc_last_error()
    rc = lib.sc_ctc_bwd_ex(fake, 0, 1, 2, 10, 8, 80, 8, fake, 3, 3, fake, fake, 0, fake, 40, 3,
                           fake, fake, fake, 0, fake, ws, null)
    assert rc == -1 and b"max_target_len + 1" in lib.sc_last_error()
    # split rows: K % 4, blank range, null pointers; B = 0 is a no-op
    rc = lib.sc_ctc_split_rows(fake, 6, null, 8, 6, fake, 3, 3, 0, fake, fake, 2, null)
    assert rc == -1 and b"16-byte" in lib.sc_last_error()
    rc = lib.sc_ctc_split_rows(fake, 8, null, 8, 8, fake, 3, 3, 8, fake, fake, 2, null)
    assert rc == -1 and b"blank" in lib.sc_last_error()
    rc = lib.sc_ctc_split_rows(null, 8, null, 8, 8, fake, 3, 3, 0, fake, fake, 2, null)
    assert rc == -1 and b"null" in lib.sc_last_error()
    assert lib.sc_ctc_split_rows(null, 8, null, 8, 8, null, 3, 3, 0, null, null, 0, null) == 0
