#!/usr/bin/env python3
"""Per-step time of the bench workload (config 2, Fst) with and without the sampled kernel events,
at the driver's step count.  usage: python tools/timing_overhead.py [steps] [reps]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
eng = Engine.get(0)
p = synth_genome(1, 1_000_000, 25, 25, seed=12345)
dev = eng.upload(p)
pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
pl.run()
pl.check()
for r in range(reps):
    for every, mask in ((0, 7), (8, 7), (8, 6), (8, 4), (16, 4)):
        pl.run_many(5)
        if every:
            pl.set_timing(steps, every=every, kernels=mask)
        pl.check()
        t0 = time.perf_counter()
        pl.run_many(steps)
        pl.check()
        dt = (time.perf_counter() - t0) / steps * 1e6
        ks = (0, 0, 0)
        if every:
            n, ks = pl.timing_read()
            pl.set_timing(0)
        print(f"steps {steps} every {every} kernels {mask}: {dt:.2f} us/step; k_scan_w {ks[2] * 1e3:.2f} us")
