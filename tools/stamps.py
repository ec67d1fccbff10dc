#!/usr/bin/env python3
"""Diagnostic: per-phase wall-clock stamps of block 0 of each kernel (needs libsfs2d_stamps.so,
built with -DSFS2D_STAMPS).  usage: SFS2D_LIB=.../libsfs2d_stamps.so python tools/stamps.py config2"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
from sfs2d import _lib as L  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "config2"
p = synth_genome(1 if which == "config2" else 32, 1_000_000 if which == "config2" else 1_562_500, 25, 25, seed=1)
eng = Engine.get(0)
dev = eng.upload(p)
pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
for _ in range(3):
    pl.run()
pl.check()
buf = (C.c_ulonglong * (64 + 2 * 4096 * 2))()
assert L.lib().sfs2d__debug_stamps(buf) == 0
t = list(buf[:64])
blk = list(buf[64:])
def d(a, b):
    return (t[b] - t[a]) * 0.01 if t[a] and t[b] else float("nan")
print(which, "K1 blk0: zero %.2f  loop %.2f  flush %.2f us" % (d(20, 21), d(21, 22), d(22, 23)))
print(which, "K2 slice0: repl+p/lp %.2f  leaves %.2f us; tail block: %.2f us" % (d(0, 1), d(1, 2), d(3, 4)))
print(which, "K3 blk0: prologue %.2f  2D pass(1st) %.2f  1D+clear %.2f  reduce+store %.2f  rest %.2f us" % (
    d(10, 11), d(11, 12), d(12, 13), d(13, 14), d(14, 15)))
print(which, "K3 fused prologue: replicas %.2f  1D+leaves %.2f  tree %.2f  logs %.2f  zero %.2f us" % (
    d(10, 16), d(16, 17), d(17, 18), d(18, 19), d(19, 11)))
print(which, "gaps: K1end->K2start %.2f  K2end->K3start %.2f us" % (d(23, 0), d(4, 10)))

# per-block spans (us) of the last run: k_prep = 0, k_scan_w = 1
import numpy as np
for k, name in ((0, "k_prep"), (1, "k_scan_w")):
    a = np.array(blk[k * 8192:(k + 1) * 8192], dtype=np.int64).reshape(4096, 2)
    a = a[(a[:, 0] > 0) & (a[:, 1] > 0)]
    if not len(a):
        continue
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) * 0.01, (a[:, 1] - t0) * 0.01
    dur = en - st
    print(which, f"{name}: blocks {len(a)}  start max {st.max():.2f}  end max {en.max():.2f}  "
          f"dur min/med/max {dur.min():.2f}/{np.median(dur):.2f}/{dur.max():.2f} us")
