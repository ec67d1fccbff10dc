#!/usr/bin/env python3
"""BASELINE config 4, scaled: R replicates x ~2,000 windows of 20 kb (Poisson-like 358.5 SNPs per
window: 717k SNPs per replicate), pop_size 50/50 (grid 101 x 101), one generation background;
the batched driver (one launch for all replicates) against the per-replicate process_window loop.
usage: python tools/sims_time.py [R] [n_pop]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
import sims_scan as S  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = int(sys.argv[2]) if len(sys.argv) > 2 else 50
ws = 20000
t0 = time.perf_counter()
reps = [synth_genome(1, 717_000, n, n, seed=1000 + i, chrom_prefix="1") for i in range(R)]
bgd = synth_genome(1, 200_000, n, n, seed=7, chrom_prefix="1")
print(f"generated {R} replicates x 717k SNPs in {time.perf_counter() - t0:.1f} s", flush=True)
bg = (S.calculate_2d_sfs(bgd, "p1", "p2", n, n, start_position=0, end_position=500000, variant_type=None),
      S.calculate_1d_sfs(bgd, "p1", n, start_position=0, end_position=500000, variant_type=None),
      S.calculate_1d_sfs(bgd, "p2", n, start_position=0, end_position=500000, variant_type=None))
S.process_windows_batch(reps[:1], *bg, ws, "p1", "p2", n, n)   # warm-up
t0 = time.perf_counter()
out = S.process_windows_batch(reps, *bg, ws, "p1", "p2", n, n)
tb = time.perf_counter() - t0
nw = sum(len(o) for o in out)
t0 = time.perf_counter()
for r in reps:
    S.process_window(r, *bg, ws, "p1", "p2", n, n, None, None, None)
tl = time.perf_counter() - t0
print(f"config4-scaled: {R} replicates, {nw} windows, grid {2*n+1}x{2*n+1}: batched {tb:.3f} s "
      f"({nw / tb:.3g} windows/s incl. upload + post-pass), per-replicate loop {tl:.3f} s ({nw / tl:.3g} windows/s)")
from sfs2d import _lib as L  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
data, _ = S._concat(reps)
eng = Engine.get(0)
dev = eng.upload(data)
pl = eng.plan(dev, ScanConfig(n1p=n, n2p=n, window=ws, bg_mode=L.BG_SUPPLIED))
pl.set_background(*S._bg_arrays(*bg, n, n))
ms, k1, k2, k3 = pl.time(5)
print(f"device time per batched run: {ms:.3f} ms (k_prep {k1:.3f}, scan {k3:.3f}): {nw / (ms * 1e-3):.3g} windows/s")
