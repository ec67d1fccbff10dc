#!/usr/bin/env python3
"""Time the multi-resolution scan (one k_prep pass, attached plans) against separate plans on the
config-3 stream: 20 kb (base, Fst) + 500 kb (Fst) + 500-SNP windows.
usage: python tools/multires_time.py [config2|config3] [iters]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
from sfs2d import _lib as L  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "config3"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
p = synth_genome(32, 1_562_500, 25, 25, seed=777) if which == "config3" else synth_genome(1, 1_000_000, 25, 25, seed=12345)
eng = Engine.get(0)
dev = eng.upload(p)
cfgs = [ScanConfig(n1p=25, n2p=25, window=20000, prev_extra=True, fst=True),
        ScanConfig(n1p=25, n2p=25, window=500000, prev_extra=True, fst=True),
        ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=500)]


def timed(run, sync):
    run()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        run()
    sync()
    return (time.perf_counter() - t0) / iters * 1e3


base = eng.plan(dev, cfgs[0])
att = [base.attach(c) for c in cfgs[1:]]
t_multi = timed(lambda: base.run(), base.check)
wins = sum(int(((pl.read()["flags"] & L.W_EMPTY) == 0).sum()) for pl in [base] + att)
base.close()
sep = [eng.plan(dev, c) for c in cfgs]
t_sep = timed(lambda: [pl.run() for pl in sep], lambda: [pl.check() for pl in sep])
print(f"{which}: {p.n} SNPs, {wins} windows at 3 resolutions: one pass {t_multi:.3f} ms, separate plans {t_sep:.3f} ms "
      f"({t_sep / t_multi:.2f}x); {wins / t_multi * 1e3:.3g} windows/s")
