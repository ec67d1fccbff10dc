#!/usr/bin/env python3
"""Per-step wall time of back-to-back config-2 runs with and without per-kernel timing events."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

p = synth_genome(1, 1_000_000, 25, 25, seed=12345)
eng = Engine.get(0)
dev = eng.upload(p)
pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000))
pl.run_many(20)
pl.check()
K = 200
for label, timing in (("no events", 0), ("events", K), ("no events", 0)):
    pl.set_timing(timing)
    pl.check()   # synchronises
    t0 = time.perf_counter()
    pl.run_many(K)
    pl.check()
    dt = (time.perf_counter() - t0) / K * 1e6
    print(f"{label:10s}: {dt:7.2f} us/step")
