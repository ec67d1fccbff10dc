#!/usr/bin/env python3
"""BASELINE config 5's precision sweep: T2D of 500-SNP windows on the asymmetric 201 x 151 grid
(pop_size 100 / 75), the reference's scipy evaluation (oracle.clr2d, fp64) against the closed form
T = 2 (sum_{x_k > 0} x_k (ln x_k - lp_k) - N ln N) evaluated
  fp32   -- every operation in float32 (counts, proportions, logs, sums)
  mixed  -- float32 log-proportion table, float64 x ln x and sums
  fp64   -- every operation in float64 (what k_scan_w / k_scan_gw compute)
and, with --gpu, the device records.  Prints max / median relative error per variant.
usage: python tools/fp_sweep.py [n_snps] [--gpu]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
sys.path.insert(0, REPO)
from oracle import sfs_oracle as O  # noqa: E402  (test infrastructure: the checker)
from sfs2d.synth import synth_genome  # noqa: E402


def closed_form(x, bg, mode):
    """T2D of one window from its inner counts x and background inner values bg."""
    lo = np.float32 if mode in ("fp32", "mixed") else np.float64
    acc = np.float32 if mode == "fp32" else np.float64
    xm = x[x > 0]
    bm = bg[x > 0]
    B = np.sum(bg.astype(lo), dtype=lo)
    lp = np.log(bm.astype(lo) / B)                      # log proportions (table precision)
    xa = xm.astype(acc)
    N = acc(xa.sum(dtype=acc))
    s = np.sum(xa * (np.log(xa) - lp.astype(acc)), dtype=acc)
    return float(acc(2) * (s - N * np.log(N)))


def sweep(n_snps=200_000, S=500, n1p=100, n2p=75, seed=5, max_windows=400):
    p = synth_genome(1, n_snps, n1p, n2p, seed=seed)
    cfg = O.Cfg(n1p, n2p)
    bg2 = O.chrom_backgrounds(p, cfg)[0][0]
    wins, _ = O.snp_windows(p, S)
    wins = wins[:: max(1, len(wins) // max_windows)]
    bgi = np.asarray(bg2).ravel()[1:-1].astype(np.float64)
    rows = []
    for w in wins:
        b, e = w[3], w[4]
        grid = O.sfs2d(p, np.arange(b, e), cfg)
        ref = O.clr2d(grid, bg2)
        if ref is None or not np.isfinite(ref):
            continue
        x = grid.ravel()[1:-1].astype(np.int64)
        rows.append((b, e, float(ref), *(closed_form(x, bgi, m) for m in ("fp32", "mixed", "fp64"))))
    return p, cfg, rows


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 200_000
    p, cfg, rows = sweep(n)
    print(f"config-5 shape: {p.n} SNPs, 500-SNP windows, grid 201 x 151, {len(rows)} windows sampled")
    for j, name in enumerate(("fp32", "mixed (fp32 lp, fp64 sums)", "fp64 closed form"), start=3):
        e = np.array([rel(r[j], r[2]) for r in rows])
        print(f"  {name:28s} max rel err {e.max():.3e}  median {np.median(e):.3e}  "
              f"windows over 1e-10: {(e > 1e-10).sum()}/{len(e)}")
    if "--gpu" in sys.argv:
        from sfs2d import _lib as L
        from sfs2d.engine import Engine, ScanConfig
        eng = Engine.get(0)
        dev = eng.upload(p)
        recs = eng.scan(dev, ScanConfig(n1p=100, n2p=75, window_mode=L.WINDOW_SNPS, window=500))
        by_b = {int(r["begin"]): float(r["t2d"]) for r in recs}
        e = np.array([rel(by_b[b], ref) for (b, _, ref, *_) in rows])
        print(f"  {'GPU (k_scan_gw, fp64)':28s} max rel err {e.max():.3e}  median {np.median(e):.3e}  "
              f"windows over 1e-10: {(e > 1e-10).sum()}/{len(e)}")


if __name__ == "__main__":
    main()
