"""ctypes binding of libsfs2d.so (include/sfs2d.h).

The library is built in-tree (``__graft_entry__.build()`` or ``make -C 2dsfs-scan_amd/csrc``).
There is no CPU fallback: if the library or a HIP device is missing, every entry point
raises ``Sfs2dError``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFS2D_LIB", os.path.join(HERE, "..", "csrc", "libsfs2d.so"))

OK = 0
E_ARG, E_HIP, E_NOMEM, E_KEY, E_GRID, E_CAP = -1, -2, -3, -4, -5, -6
WINDOW_BP, WINDOW_SNPS = 0, 1
BG_PER_CHROM, BG_SUPPLIED = 0, 1
F_PREV_EXTRA = 1
F_FST = 2
W_EMPTY = 0x80000000
W_BG2_ZERO, W_BG1A_ZERO, W_BG1B_ZERO = 0x1, 0x2, 0x4
W_EXTRA = 0x40000000


def bg_row_words(n1p: int, n2p: int) -> int:
    """SFS2D_BG_ROW_WORDS: one background as an int64 row [2D bins | unfolded pop-1 | unfolded pop-2 |
    inner 2D sum] (sfs2d_bg_hist_dev, sfs2d_plan_bg_rows_dev)."""
    return (2 * n1p + 1) * (2 * n2p + 1) + 2 * n1p + 2 * n2p + 3

# the exported symbols of include/sfs2d.h (checked by tests/test_lib_abi.py)
EXPORTS = [
    "sfs2d_abi_version", "sfs2d_ctx_create", "sfs2d_ctx_destroy", "sfs2d_last_error", "sfs2d_ctx_set_stream",
    "sfs2d_data_upload", "sfs2d_data_wrap_device", "sfs2d_data_free", "sfs2d_bg_hist", "sfs2d_plan_create",
    "sfs2d_plan_num_records", "sfs2d_plan_set_background", "sfs2d_plan_run", "sfs2d_plan_run_many", "sfs2d_plan_set_timing_sampled",
    "sfs2d_plan_set_timing_kernels",
    "sfs2d_plan_fst_read", "sfs2d_plan_fst_buffer", "sfs2d_plan_read",
    "sfs2d_plan_bg_buffer", "sfs2d_plan_bg_words", "sfs2d_plan_bg_exchange", "sfs2d_plan_run_phase", "sfs2d_plan_check", "sfs2d_plan_time",
    "sfs2d_plan_destroy", "sfs2d_scan", "sfs2d_plan_set_timing", "sfs2d_plan_timing_read",
    "sfs2d_plan_stats", "sfs2d_plan_grids", "sfs2d_plan_scan_kernel", "sfs2d_plan_attach", "sfs2d_data_synth_sims",
    "sfs2d_data_read", "sfs2d_plan_run_streams", "sfs2d_ctx_use_own_stream", "sfs2d_bg_hist_dev", "sfs2d_plan_bg_rows_dev", "sfs2d_plan_bg_rows_set_dev",
    "sfs2d_ctx_get_stream", "sfs2d_plan_set_fst_out", "sfs2d_graph_create", "sfs2d_graph_launch", "sfs2d_graph_destroy",
]
ABI_VERSION = 2   # SFS2D_ABI_VERSION of include/sfs2d.h


class Sfs2dError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"sfs2d error {code}: {msg}")
        self.code = code


class SynthParams(C.Structure):   # sfs2d_synth_params
    _fields_ = [("seed", C.c_uint64), ("generation", C.c_uint32), ("n_replicates", C.c_uint32),
                ("n_windows", C.c_uint32), ("window_bp", C.c_uint32), ("n1p", C.c_int32), ("n2p", C.c_int32)]


class Params(C.Structure):
    _fields_ = [
        ("n1p", C.c_int32), ("n2p", C.c_int32), ("fold", C.c_int32), ("window_mode", C.c_int32),
        ("window", C.c_int64), ("bg_mode", C.c_int32), ("ann_want", C.c_int32),
        ("has_start", C.c_int32), ("has_end", C.c_int32), ("start_pos", C.c_int64), ("end_pos", C.c_int64),
        ("flags", C.c_uint32), ("scan_wgs_per_cu", C.c_uint32),
    ]


WINDOW_DTYPE = np.dtype([
    ("chrom", "<u4"), ("wid", "<u4"), ("begin", "<u4"), ("end", "<u4"), ("snp_count", "<u4"),
    ("n2", "<u4"), ("n2_all", "<u4"), ("n1a", "<u4"), ("n1b", "<u4"), ("flags", "<u4"),
    ("t2d", "<f8"), ("t1d_p1", "<f8"), ("t1d_p2", "<f8"),
])
assert WINDOW_DTYPE.itemsize == 64

_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise Sfs2dError(E_ARG, f"HIP library not built: {os.path.abspath(LIB_PATH)} missing "
                                "(run __graft_entry__.build() or make -C 2dsfs-scan_amd/csrc)")
    # one HIP runtime per process: torch's wheel bundles libamdhip64 (soname libamdhip64.so.7, which
    # torch itself needs as "libamdhip64.so"); if this library loaded /opt/rocm's copy first, a later
    # torch import would bring a second runtime that finds no GPU.  Loaded after torch, this
    # library's libamdhip64.so.7 resolves to torch's copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(os.path.abspath(LIB_PATH))
    vp, i32, i64, u32p = C.c_void_p, C.c_int32, C.c_int64, C.POINTER(C.c_uint32)
    L.sfs2d_abi_version.restype = C.c_int
    v = L.sfs2d_abi_version()
    if v != ABI_VERSION and not (v < 0 and os.environ.get("SFS2D_ALLOW_ABLATION") == "1"):
        raise Sfs2dError(E_ARG, f"{os.path.abspath(LIB_PATH)}: ABI version {v}, expected {ABI_VERSION}"
                                + (" (an ablation build: timing only, wrong results)" if v < 0 else ""))
    L.sfs2d_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.sfs2d_ctx_destroy.argtypes = [vp]
    L.sfs2d_last_error.argtypes = [vp]
    L.sfs2d_last_error.restype = C.c_char_p
    L.sfs2d_ctx_set_stream.argtypes = [vp, vp]
    L.sfs2d_data_upload.argtypes = [vp, vp, vp, vp, i64, vp, i32, C.POINTER(vp)]
    L.sfs2d_data_wrap_device.argtypes = [vp, vp, vp, vp, i64, vp, vp, i32, C.POINTER(vp)]
    L.sfs2d_data_free.argtypes = [vp]
    L.sfs2d_bg_hist.argtypes = [vp, vp, C.POINTER(Params), i32, vp, vp, vp]
    L.sfs2d_plan_create.argtypes = [vp, vp, C.POINTER(Params), C.POINTER(vp)]
    L.sfs2d_plan_num_records.argtypes = [vp]
    L.sfs2d_plan_num_records.restype = i64
    L.sfs2d_plan_set_background.argtypes = [vp, vp, vp, vp]
    L.sfs2d_plan_run.argtypes = [vp, vp]
    L.sfs2d_plan_run_many.argtypes = [vp, C.c_int, vp]
    L.sfs2d_plan_run_streams.argtypes = [vp, vp, vp, C.c_int, C.c_int]
    L.sfs2d_graph_create.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.POINTER(vp)]
    L.sfs2d_graph_launch.argtypes = [vp, C.c_int]
    L.sfs2d_graph_destroy.argtypes = [vp]
    L.sfs2d_plan_set_timing_sampled.argtypes = [vp, C.c_int, C.c_int]
    L.sfs2d_plan_set_timing_kernels.argtypes = [vp, C.c_int, C.c_int, C.c_int]
    L.sfs2d_plan_fst_read.argtypes = [vp, vp, i64]
    L.sfs2d_plan_fst_buffer.argtypes = [vp, C.POINTER(vp), C.POINTER(i64)]
    L.sfs2d_plan_run_phase.argtypes = [vp, C.c_int, vp]
    L.sfs2d_plan_read.argtypes = [vp, vp, i64, C.POINTER(i64)]
    L.sfs2d_plan_bg_buffer.argtypes = [vp, C.POINTER(vp), C.POINTER(i64)]
    L.sfs2d_plan_bg_words.argtypes = [vp, C.POINTER(i64), C.POINTER(i64), C.POINTER(i64)]
    L.sfs2d_plan_bg_exchange.argtypes = [vp, vp, vp, C.c_int]
    L.sfs2d_bg_hist_dev.argtypes = [vp, vp, C.POINTER(Params), i32, vp]
    L.sfs2d_plan_bg_rows_dev.argtypes = [vp, vp, i64]
    L.sfs2d_plan_bg_rows_set_dev.argtypes = [vp, vp, i64]
    L.sfs2d_plan_check.argtypes = [vp]
    L.sfs2d_plan_time.argtypes = [vp, C.c_int] + [C.POINTER(C.c_double)] * 4
    L.sfs2d_plan_destroy.argtypes = [vp]
    L.sfs2d_plan_set_timing.argtypes = [vp, C.c_int]
    L.sfs2d_plan_stats.argtypes = [vp, C.POINTER(C.c_uint32)]
    L.sfs2d_plan_grids.argtypes = [vp, C.POINTER(i64), C.POINTER(i64)]
    L.sfs2d_plan_scan_kernel.argtypes = [vp]
    L.sfs2d_plan_scan_kernel.restype = C.c_char_p
    L.sfs2d_plan_attach.argtypes = [vp, C.POINTER(Params), C.POINTER(vp)]
    L.sfs2d_data_synth_sims.argtypes = [vp, C.POINTER(SynthParams), vp, vp, i32, vp, i32, C.POINTER(vp)]
    L.sfs2d_data_read.argtypes = [vp, vp, vp, i64]
    L.sfs2d_ctx_use_own_stream.argtypes = [vp]
    L.sfs2d_ctx_get_stream.argtypes = [vp, C.POINTER(vp)]
    L.sfs2d_plan_set_fst_out.argtypes = [vp, vp]
    L.sfs2d_plan_timing_read.argtypes = [vp, C.POINTER(C.c_int)] + [C.POINTER(C.c_double)] * 3
    L.sfs2d_scan.argtypes = [vp, vp, C.POINTER(Params), vp, vp, vp, vp, i64, C.POINTER(i64)]
    _lib = L
    return L


def ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None
