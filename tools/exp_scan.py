#!/usr/bin/env python3
"""A/B timings of the config-3 scan (5e7 SNPs, 20 kb, Fst) under environment settings read at plan
creation (SFS2D_WGS: scan workgroups in the grid; SFS2D_FUSED ...) and, with SFS2D_LIB_VARIANTS, under
other builds of the library (one subprocess each).  Prints per-variant k_prep / k_scan_w times (HIP
events in the dispatch packets, one stream).
usage: python tools/exp_scan.py [config2|config3] [ENV=VAL[,ENV=VAL]] ...   (each arg one variant; a
"nofst" item in a variant scans without Fst, compared with the first variant's records only)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))

import numpy as np  # noqa: E402
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "config3"
variants = sys.argv[2:] or ["-"]
if which == "config2":
    p = synth_genome(1, 1_000_000, 25, 25, seed=12345)
else:
    p = synth_genome(32, 1_562_500, 25, 25, seed=777)
eng = Engine.get(0)
dev = eng.upload(p)
ref = None
for rep in range(2):
    for v in variants:
        env = dict(kv.split("=", 1) for kv in v.split(",") if "=" in kv)
        fst_on = "nofst" not in v.split(",")
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=fst_on))
        for k, o in old.items():
            if o is None:
                os.environ.pop(k)
            else:
                os.environ[k] = o
        pl.run()
        pl.check()
        recs = pl.read()
        fst = pl.read_fst() if fst_on else ref[1] if ref else None
        if ref is None:
            ref = (recs, fst)
        same = recs.tobytes() == ref[0].tobytes()
        ints = all(np.array_equal(recs[f], ref[0][f]) for f in ("chrom", "wid", "begin", "end", "snp_count", "n2", "n1a", "n1b", "flags"))
        rel = 0.0
        for f in ("t2d", "t1d_p1", "t1d_p2"):
            a, b = recs[f], ref[0][f]
            m = np.isfinite(b) & (b != 0)
            rel = max(rel, float(np.max(np.abs(a[m] - b[m]) / np.abs(b[m]))) if m.any() else 0.0)
        fm = np.isfinite(ref[1]) & (ref[1] != 0)
        frel = float(np.max(np.abs(fst[fm] - ref[1][fm]) / np.abs(ref[1][fm]))) if fm.any() else 0.0
        pl.set_timing(12, every=1)
        pl.run_many(12)
        _, (k1, k2, k3) = pl.timing_read()
        pl.set_timing(0)
        print(f"{which} rep {rep} {v:40s} [{pl.scan_kernel()}] k_prep {k1 * 1e3:8.1f} us  k_bg_slice {k2 * 1e3:6.1f}  k_scan_w {k3 * 1e3:8.1f} us"
              f"  grid {pl.grids()[1] // 512} WGs  bytes-same={same} ints={ints} rel={rel:.1e} fst_rel={frel:.1e}"
              f"  exact={pl.stats()}", flush=True)
        pl.close()
