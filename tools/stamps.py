#!/usr/bin/env python3
"""Diagnostic: per-phase wall-clock stamps of block 0 of each kernel (needs libsfs2d_stamps.so,
built with -DSFS2D_STAMPS).  usage: SFS2D_LIB=.../libsfs2d_stamps.so python tools/stamps.py config2|config3 [chromosomes]|config5"""
import ctypes as C
import numpy as np
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
from sfs2d import _lib as L  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "config2"
if which in ("config5", "config5b"):   # 201 x 151 grid, 500-SNP windows (large-grid kernels, k_bg_slice with its tail)
    # config5b: the bench's shape, 4 chromosomes x 250,000 SNPs (4 backgrounds)
    p = synth_genome(1, 1_000_000, 100, 75, seed=55) if which == "config5" else synth_genome(4, 250_000, 100, 75, seed=2024)
    cfg = ScanConfig(n1p=100, n2p=75, window_mode=L.WINDOW_SNPS, window=500)
else:
    nch = int(sys.argv[2]) if len(sys.argv) > 2 else 32   # config3 [chromosomes]: a rank's share
    p = synth_genome(1 if which == "config2" else nch, 1_000_000 if which == "config2" else 1_562_500, 25, 25, seed=1)
    cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=True, scan_wgs_per_cu=1 if which == "config3" else 0)
eng = Engine.get(0)
dev = eng.upload(p)
pl = eng.plan(dev, cfg)
for _ in range(3):
    pl.run()
pl.check()
buf = (C.c_ulonglong * (64 + 2 * 4096 * 2 + 4096 * 8 * 2 + 1024 * 2))()
assert L.lib().sfs2d__debug_stamps(buf) == 0
t = list(buf[:64])
blk = list(buf[64:64 + 16384])
wvs = np.array(buf[64 + 16384:64 + 16384 + 65536], dtype=np.int64).reshape(4096 * 8, 2)
bgs = np.array(buf[64 + 16384 + 65536:], dtype=np.int64).reshape(1024, 2)
def d(a, b):
    return (t[b] - t[a]) * 0.01 if t[a] and t[b] else float("nan")
print(which, "K1 blk0: zero %.2f  loop %.2f  flush %.2f us" % (d(20, 21), d(21, 22), d(22, 23)))
print(which, "K2 slice0: repl+p/lp %.2f  leaves %.2f us; slice0 end -> tail start %.2f us; tail block: %.2f us" % (
    d(0, 1), d(1, 2), d(2, 3), d(3, 4)))
print(which, "K3 blk0: prologue %.2f  2D pass(1st) %.2f  1D+clear %.2f  reduce+store %.2f  rest %.2f us" % (
    d(10, 11), d(11, 12), d(12, 13), d(13, 14), d(14, 15)))
print(which, "K3 fused prologue: replicas %.2f  1D+leaves %.2f  tree %.2f  logs %.2f  zero %.2f us" % (
    d(10, 16), d(16, 17), d(17, 18), d(18, 19), d(19, 11)))
print(which, "K3 sliced prologue: D/F copy %.2f  lp copy %.2f  leaf tree %.2f  head %.2f  zero %.2f us" % (
    d(10, 24), d(24, 25), d(25, 26), d(26, 27), d(27, 11)))
nb_s = int((bgs[:, 0] > 0).sum())
if nb_s:   # k_bg_slice blocks (x + y * gridDim.x): start and work-done times from the earliest start
    g0 = bgs[:nb_s, 0].min()
    st_s, en_s = (bgs[:nb_s, 0] - g0) * 0.01, (bgs[:nb_s, 1] - g0) * 0.01
    slow = np.argsort(en_s)[-6:]
    print(which, f"k_bg_slice: blocks {nb_s}  start max {st_s.max():.2f}  done p50/max {np.median(en_s):.2f}/{en_s.max():.2f} us;"
          " latest blocks (index: start-done):", " ".join(f"{i}:{st_s[i]:.1f}-{en_s[i]:.1f}" for i in slow))
print(which, "gaps: K1end->K2start %.2f  K2end->K3start %.2f us" % (d(23, 0), d(4, 10)))

# per-block spans (us) of the last run: k_prep = 0, k_scan_w = 1
import numpy as np
for k, name in ((0, "k_prep"), (1, "k_scan_w")):
    a = np.array(blk[k * 8192:(k + 1) * 8192], dtype=np.int64).reshape(4096, 2)
    ids = np.nonzero((a[:, 0] > 0) & (a[:, 1] > 0))[0]
    a = a[ids]
    if not len(a):
        continue
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) * 0.01, (a[:, 1] - t0) * 0.01
    dur = en - st
    print(which, f"{name}: blocks {len(a)}  start max {st.max():.2f}  end max {en.max():.2f}  "
          f"dur min/med/max {dur.min():.2f}/{np.median(dur):.2f}/{dur.max():.2f} us")
    # end time by blockIdx % 8 (the usual XCD round robin)
    print(which, f"{name}: end by block%8 (mean/max):",
          " ".join(f"{en[ids % 8 == x].mean():.0f}/{en[ids % 8 == x].max():.0f}" for x in range(8)))
    q = np.percentile(en, [10, 50, 90])
    print(which, f"{name}: end p10/p50/p90 {q[0]:.1f}/{q[1]:.1f}/{q[2]:.1f} us")

# k_scan_w per wavefront: windows scanned and end time; per chromosome (blocks grouped by chunk order)
nb = len([1 for i in range(4096) if blk[8192 + 2 * i] > 0])
w = wvs[: nb * 8]
live = w[:, 0] > 0
t0 = np.array(blk[8192:8192 + 2 * nb:2], dtype=np.int64).min()
en = (w[:, 0] - t0) * 0.01
print(which, f"k_scan_w waves: {live.sum()}  windows/wave min/med/max {w[live,1].min()}/{int(np.median(w[live,1]))}/{w[live,1].max()}"
      f"  end min/med/max {en[live].min():.1f}/{np.median(en[live]):.1f}/{en[live].max():.1f} us")
if which != "config2":
    # workgroups are interleaved over the grid: block b scans chromosome b % 32 (equal chromosomes)
    nc = {"config5": 32, "config5b": 4}.get(which) or nch
    chrom = (np.arange(nb * 8) // 8) % nc
    ce = [(en[chrom == c].min(), en[chrom == c].max(), int(w[chrom == c, 1].sum())) for c in range(nc)]
    print(which, "per chromosome end min-max / windows:", " ".join(f"{a:.0f}-{b:.0f}/{n}" for a, b, n in ce))
