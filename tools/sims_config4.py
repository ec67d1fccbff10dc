#!/usr/bin/env python3
"""BASELINE config 4 on one GPU with replicates generated in HBM: G generations x R replicates x
2,000 windows of 20 kb, Poisson(358.5) SNPs per window, pop_size 50/50 (101 x 101 grid, the
workgroup-per-window path).  Per generation: generate (k_synth_sims), background = all the
generation's SNPs with pos in [0, 500000] (sims_scan.py:615-617: 2D folded, 1D unfolded, read at
keys 1..n-1), one supplied-background plan over all replicates, scan; records stay on the device.
usage: python tools/sims_config4.py [replicates_per_generation] [generations] [runs]"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
import sims_scan as S  # noqa: E402
from sfs2d import _lib as L  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import miss_table, sims_window_counts  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 2500
G = int(sys.argv[2]) if len(sys.argv) > 2 else 4
runs = int(sys.argv[3]) if len(sys.argv) > 3 else 3
n, nwin, ws, seed = 50, 2000, 20000, 20251016
eng = Engine.get(0)
mt = miss_table(2 * n)
tot_w, tot_snp, t_gen, t_scan, t_bg = 0, 0, 0.0, 0.0, 0.0
for g in range(G):
    wc = sims_window_counts(seed, g, R, nwin)
    nsnp = int(wc.astype(np.int64).sum())
    t0 = time.perf_counter()
    dev = eng.synth_sims(seed, g, R, nwin, ws, n, n, wc, mt, mt)
    t1 = time.perf_counter()
    h2, u1, u2 = eng.bg_hist(dev, ScanConfig(n1p=n, n2p=n, start_position=0, end_position=500000), -1)
    b2 = h2.reshape(-1).astype(np.float64)
    bg = (b2, u1[: n + 1].astype(np.float64), u2[: n + 1].astype(np.float64))   # unfolded 1D (quirk Q7)
    t2 = time.perf_counter()
    pl = eng.plan(dev, ScanConfig(n1p=n, n2p=n, window=ws, bg_mode=L.BG_SUPPLIED))
    pl.set_background(*bg)
    pl.run()
    pl.check()
    ms, k1, k2, k3 = pl.time(runs)
    recs = pl.read()
    nw = int(((recs["flags"] & L.W_EMPTY) == 0).sum())
    pl.close()
    dev.close()
    tot_w += nw
    tot_snp += nsnp
    t_gen += t1 - t0
    t_bg += t2 - t1
    t_scan += ms * 1e-3
    print(f"generation {g}: {R} replicates, {nsnp} SNPs ({nsnp * 8 / 1e9:.1f} GB packed), {nw} windows: "
          f"generate {t1 - t0:.2f} s, background {t2 - t1:.2f} s, scan {ms:.2f} ms per run "
          f"(k_prep {k1:.2f}, scan kernel {k3:.2f}) = {nw / (ms * 1e-3):.3g} windows/s", flush=True)
print(f"config 4 ({G} x {R} replicates): {tot_w} windows, {tot_snp} SNPs; device scan time {t_scan:.3f} s "
      f"= {tot_w / t_scan:.3g} windows/s; generation {t_gen:.1f} s, backgrounds {t_bg:.1f} s")
