"""ctypes binding of the C oracle (oracle/sfs_oracle_c.c, built by `make -C oracle`).

TEST INFRASTRUCTURE ONLY: tests/ and bench.py's cpu_baseline leg use it (the baseline is this
restatement timed on the host's cores).  The product path never imports it."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libsfs_oracle_c.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = C.CDLL(LIB_PATH)
        vp, i64 = C.c_void_p, C.c_int64
        L.oracle_scan_bp.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_int, i64,
                                     C.POINTER(i64), vp, vp, vp, vp, vp, vp, vp]
        L.oracle_scan_bp.restype = C.c_int
        L.oracle_max_threads.restype = C.c_int
        _lib = L
    return _lib


def max_threads() -> int:
    return lib().oracle_max_threads()


def scan_bp(p, ws: int, n1p: int, n2p: int, threads: int = 0):
    """Fixed-bp windows with per-chromosome backgrounds (combined_scan's per-window statistics,
    before the host quirks Q6 / Q9).  Returns a dict of numpy arrays: chrom, start, b, e, T2D,
    T1D_p1, T1D_p2 (NaN = None)."""
    L = lib()
    counts = np.ascontiguousarray(p.counts, dtype=np.uint32)
    pos = np.ascontiguousarray(p.pos, dtype=np.uint32)
    off = np.ascontiguousarray(p.chrom_off, dtype=np.int64)
    cap = int(len(counts) + 2 * len(off) + 16)
    out = {"chrom": np.zeros(cap, np.int32), "start": np.zeros(cap, np.uint32), "b": np.zeros(cap, np.int64),
           "e": np.zeros(cap, np.int64), "T2D": np.zeros(cap), "T1D_p1": np.zeros(cap), "T1D_p2": np.zeros(cap)}
    n = C.c_int64()
    rc = L.oracle_scan_bp(counts.ctypes.data, pos.ctypes.data, off.ctypes.data, len(off) - 1, n1p, n2p, ws,
                          int(threads), cap, C.byref(n), *(out[k].ctypes.data for k in
                                                           ("chrom", "start", "b", "e", "T2D", "T1D_p1", "T1D_p2")))
    if rc != 0:
        raise RuntimeError(f"oracle_scan_bp failed ({rc}, {n.value} windows)")
    return {k: v[: n.value] for k, v in out.items()}
