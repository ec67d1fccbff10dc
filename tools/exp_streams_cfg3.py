#!/usr/bin/env python3
"""Config 3 (5e7 SNPs, 32 chromosomes, 20 kb, Fst) passes: one plan back to back vs S plans on S HIP
streams (independent passes overlapping: one pass's bandwidth-bound k_prep beside the previous
pass's compute-bound k_scan_w).  With a chromosome count below 32, one rank's share of the strong-scaling
bench (32 / N chromosomes per rank at N GPUs).
usage: python tools/exp_streams_cfg3.py [runs] [fst|nofst] [scan workgroups per CU] [chromosomes]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))

import torch  # noqa: E402

from sfs2d.engine import Engine, Plan, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 24
fst = len(sys.argv) > 2 and sys.argv[2] == "fst"
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 0
nchr = int(sys.argv[4]) if len(sys.argv) > 4 else 32
p = synth_genome(32, 1_562_500, 25, 25, seed=777)
if nchr < 32:
    p = p.subset_chroms(list(range(nchr)))
eng = Engine.get(0)
s0 = torch.cuda.Stream()
eng.set_stream(s0.cuda_stream)
dev = eng.upload(p)
cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=fst, scan_wgs_per_cu=cap)
plans = [eng.plan(dev, cfg) for _ in range(4)]
streams = [s0.cuda_stream] + [torch.cuda.Stream().cuda_stream for _ in range(3)]
nrec = plans[0].nrec
outs = [torch.zeros((nrec, 64), dtype=torch.uint8, device="cuda:0") for _ in range(4)]
nwin = None
t_s = time.perf_counter()
while time.perf_counter() - t_s < 0.3:   # device settle (as bench.py)
    Plan.run_streams(plans[:2], streams[:2], 16, [o.data_ptr() for o in outs[:2]])
    torch.cuda.synchronize()
for S in (1, 2, 3, 1, 2):
    Plan.run_streams(plans[:S], streams[:S], 2 * S, [o.data_ptr() for o in outs[:S]])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Plan.run_streams(plans[:S], streams[:S], runs, [o.data_ptr() for o in outs[:S]])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / runs
    for k in range(1, S):
        assert torch.equal(outs[k], outs[0])
    if nwin is None:
        from sfs2d import _lib as L
        import numpy as np
        r = np.frombuffer(outs[0].cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
        nwin = int(((r["flags"] & L.W_EMPTY) == 0).sum())
    print(f"{nchr} chromosomes, streams {S}: {dt * 1e3:.4f} ms per pass, {nwin / dt:.3e} windows/s, "
          f"{(12 * p.n + 64 * nwin) / dt / 1e12:.2f} TB/s (SURVEY 8d bytes)", flush=True)
