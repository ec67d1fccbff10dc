#!/usr/bin/env python3
"""One config-3 scan (5e7 SNPs, 32 chromosomes, 20 kb, Fst) as a user runs it once: the whole genome as
one plan (k_prep then k_scan_w in series on one stream) vs the genome cut into K chromosome groups, one
plan each, the groups alternating over 2 HIP streams (sfs2d_plan_run_streams, first run phase-split), so
that group i's k_scan_w overlaps group i+1's k_prep inside ONE pass.  Per-chromosome backgrounds make the
groups independent (no exchange).  Each pass is enqueued, then synchronised, so no pass overlaps the
next; the groups' records are checked equal to the whole plan's (chromosome ids group-local).
usage: python tools/exp_chunked_pass.py [passes] [caps, e.g. 0,1]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from sfs2d import _lib as L  # noqa: E402
from sfs2d.engine import Engine, Plan, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 30
caps = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,1").split(",")]
p = synth_genome(32, 1_562_500, 25, 25, seed=777)
eng = Engine.get(0)
s0 = torch.cuda.Stream()
eng.set_stream(s0.cuda_stream)
streams = [s0.cuda_stream, torch.cuda.Stream().cuda_stream]
dev = eng.upload(p)


def recs(t):
    return np.frombuffer(t.cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)


def timed(fn, n):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3, float(np.min(ts)) * 1e3


whole = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
wout = torch.zeros((whole.nrec, 64), dtype=torch.uint8, device="cuda:0")
t_s = time.perf_counter()
while time.perf_counter() - t_s < 0.3:   # device settle (as bench.py)
    whole.run_many(8, wout.data_ptr())
    torch.cuda.synchronize()
ref = recs(wout)
live = (ref["flags"] & L.W_EMPTY) == 0
print(f"whole genome, one plan: {timed(lambda: whole.run(wout.data_ptr()), R)} ms (median, min) per pass", flush=True)
for cap in caps:
    for K in (2, 4, 8, 16):
        groups = np.array_split(np.arange(32), K)
        subs = [p.subset_chroms(g.tolist()) for g in groups]
        devs = [eng.upload(s) for s in subs]
        cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=True, scan_wgs_per_cu=cap)
        plans = [eng.plan(d, cfg) for d in devs]
        outs = [torch.zeros((q.nrec, 64), dtype=torch.uint8, device="cuda:0") for q in plans]
        ptrs = [o.data_ptr() for o in outs]
        sk = [streams[i % 2] for i in range(K)]
        fn = lambda: Plan.run_streams(plans, sk, K, ptrs)  # noqa: E731
        med, mn = timed(fn, R)
        parts = []
        for g, o in zip(groups, outs):   # begin / end are SNP indices into the group's own data
            r = recs(o)
            r = r[(r["flags"] & L.W_EMPTY) == 0].copy()
            r["begin"] += np.uint32(p.chrom_off[g[0]])
            r["end"] += np.uint32(p.chrom_off[g[0]])
            parts.append(r)
        got = np.concatenate(parts)
        exp = ref[live]
        ok = (len(got) == len(exp) and all(np.array_equal(got[f], exp[f]) for f in
                                           ("wid", "begin", "end", "snp_count", "n2", "n1a", "n1b", "flags"))
              and all(np.array_equal(got[f].view(np.uint64), exp[f].view(np.uint64)) for f in
                      ("t2d", "t1d_p1", "t1d_p2")))
        print(f"cap {cap}, {K} groups on 2 streams: {med:.4f} ms median, {mn:.4f} min per pass; "
              f"records equal to the whole plan's: {ok}", flush=True)
        for q in plans:
            q.close()
        for d in devs:
            d.close()
whole.close()
dev.close()
