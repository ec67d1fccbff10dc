#!/usr/bin/env python3
"""Median k_prep / scan kernel times of config 3 (5e7 SNPs, 20 kb, Fst) under the library SFS2D_LIB
(A/B of builds: one process per library).  usage: SFS2D_LIB=... python tools/ktime.py [fst|nofst] [reps] [config3|config2]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
import numpy as np  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

fst = (sys.argv[1] if len(sys.argv) > 1 else "fst") == "fst"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
which = sys.argv[3] if len(sys.argv) > 3 else "config3"
p = synth_genome(32, 1_562_500, 25, 25, seed=777) if which == "config3" else synth_genome(1, 1_000_000, 25, 25, seed=12345)
eng = Engine.get(0)
dev = eng.upload(p)
pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=fst))
pl.run_many(40)
pl.check()
k1s, k3s = [], []
for _ in range(reps):
    pl.set_timing(12, every=1)
    pl.run_many(12)
    _, (k1, _, k3) = pl.timing_read()
    pl.set_timing(0)
    k1s.append(k1 * 1e3)
    k3s.append(k3 * 1e3)
import time  # noqa: E402
pl.check()
t0 = time.perf_counter()
pl.run_many(200)
pl.check()
pass_us = (time.perf_counter() - t0) / 200 * 1e6
import hashlib  # noqa: E402
digest = hashlib.sha1(pl.read().tobytes() + (pl.read_fst().tobytes() if fst else b"")).hexdigest()[:12]
print(f"{os.path.basename(os.environ.get('SFS2D_LIB', 'libsfs2d.so'))} {which} fst={fst} [{pl.scan_kernel()}] k_prep median {np.median(k1s):.1f} us"
      f"  scan median {np.median(k3s):.1f} us  (min {min(k3s):.1f} max {max(k3s):.1f})  pass {pass_us:.1f} us  out {digest}", flush=True)
