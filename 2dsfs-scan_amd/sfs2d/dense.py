"""calculate_likelihood_2D / _1D on dense SFS dicts, evaluated by the HIP scan kernel.

The reference's primitives (twoDSFS_class.py:478-537, 625-684; sims_scan.py:325-440) take a
foreground SFS dict and a background dict.  Rather than a second implementation of the
statistic, the foreground spectrum is turned into a synthetic SNP stream (one SNP per count,
no fold, alt counts = the bin coordinates) scanned as ONE fixed-SNP window against the supplied
background -- the same kernel and the same value semantics as the window scans.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .engine import ScanConfig
from .pack import PackedSNPs, pack_counts


def _one_window(eng, a1, a2, n1p, n2p, bg2d, bg1a, bg1b):
    n = len(a1)
    counts = pack_counts(2 * n1p - a1, a1, 2 * n2p - a2, a2)
    p = PackedSNPs(counts, np.arange(1, n + 1, dtype=np.uint32), np.array([0, n], np.int64), ["fg"],
                   np.zeros(n, np.uint16), ["x"], "p1", "p2")
    cfg = ScanConfig(n1p=n1p, n2p=n2p, fold=False, window_mode=L.WINDOW_SNPS, window=n, bg_mode=L.BG_SUPPLIED)
    dev = eng.upload(p)
    try:
        recs = eng.scan(dev, cfg, (bg2d, bg1a, bg1b))
    finally:
        dev.close()
    return recs[0]


def clr_2d(eng, fg: dict, bg: dict, guards=True):
    bins = sorted(fg.keys())
    inner = bins[1:-1]
    counts_fg = [int(fg[k]) for k in inner]
    total_fg = sum(counts_fg)
    if total_fg == 0:
        if guards:
            return None
        raise ZeroDivisionError("division by zero")
    counts_bg = [bg[k] for k in inner]
    if sum(counts_bg) == 0:
        if guards:
            return None
        raise ZeroDivisionError("division by zero")
    n1, n2 = bins[-1]
    grid = [(i, j) for i in range(n1 + 1) for j in range(n2 + 1)]
    if n1 % 2 or n2 % 2 or bins != grid:
        raise NotImplementedError("calculate_likelihood_2D on a non-standard SFS grid")
    n1p, n2p = n1 // 2, n2 // 2
    a1 = np.repeat(np.array([k[0] for k in inner], np.int64), counts_fg)
    a2 = np.repeat(np.array([k[1] for k in inner], np.int64), counts_fg)
    bg2 = np.zeros(len(grid), np.float64)
    bg2[1:-1] = np.array(counts_bg, dtype=np.float64)
    r = _one_window(eng, a1, a2, n1p, n2p, bg2, np.ones(n1p + 1), np.ones(n2p + 1))
    return float(r["t2d"])


def clr_1d(eng, fg: dict, bg: dict, guards=True):
    bins = sorted(fg.keys())
    inner = bins[1:-1]
    counts_fg = [int(fg[k]) for k in inner]
    total_fg = sum(counts_fg)
    if total_fg == 0:
        if guards:
            return None
        raise ZeroDivisionError("division by zero")
    counts_bg = [bg[k] for k in inner]
    if sum(counts_bg) == 0:
        if guards:
            return None
        raise ZeroDivisionError("division by zero")
    n = bins[-1]
    if bins != list(range(n + 1)):
        raise NotImplementedError("calculate_likelihood_1D on a non-standard folded SFS")
    a1 = np.repeat(np.array(inner, np.int64), counts_fg)
    a2 = np.zeros_like(a1)
    b1 = np.zeros(n + 1, np.float64)
    b1[1:n] = np.array(counts_bg, dtype=np.float64)
    r = _one_window(eng, a1, a2, n, n, np.ones((2 * n + 1) ** 2), b1, np.ones(n + 1))
    return float(r["t1d_p1"])
