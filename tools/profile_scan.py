#!/usr/bin/env python3
"""Run one scan configuration a few times (no torch) -- the target of rocprofv3 kernel-trace / PMC runs.

usage: python tools/profile_scan.py [config2|config3|config5] [iters] [fst]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))

from sfs2d import _lib as L  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "config3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
fst = len(sys.argv) > 3 and sys.argv[3] == "fst"
if which == "config2":
    p, cfg = synth_genome(1, 1_000_000, 25, 25, seed=12345), ScanConfig(n1p=25, n2p=25, window=20000)
elif which == "config3":
    p, cfg = synth_genome(32, 1_562_500, 25, 25, seed=777), ScanConfig(n1p=25, n2p=25, window=20000)
else:
    p = synth_genome(1, 1_000_000, 100, 75, seed=55)
    cfg = ScanConfig(n1p=100, n2p=75, window_mode=L.WINDOW_SNPS, window=500)
cfg.fst = fst
eng = Engine.get(0)
dev = eng.upload(p)
pl = eng.plan(dev, cfg)
pl.run()
pl.check()
pl.set_timing(iters)
t0 = time.perf_counter()
for _ in range(iters):
    pl.run()
n, ks = pl.timing_read()
print(which, "nrec", pl.nrec, "k1/k2/k3 ms", ks, "exact-path windows", pl.stats(), "wall/iter ms",
      (time.perf_counter() - t0) / iters * 1e3)
