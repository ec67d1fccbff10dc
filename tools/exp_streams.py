#!/usr/bin/env python3
"""Independent passes overlapped on S HIP streams (sfs2d_plan_run_streams) with the scan kernel capped at
W workgroups per CU (sfs2d_params.scan_wgs_per_cu; 0 = all that fit), per pass time and windows/s.
usage: python tools/exp_streams.py config2|config3 runs fst|nofst "S,W S,W ..." """
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")

import torch  # noqa: E402

from sfs2d.engine import Engine, Plan, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

which, runs, fst = sys.argv[1], int(sys.argv[2]), sys.argv[3] == "fst"
combos = [tuple(int(x) for x in c.split(",")) for c in sys.argv[4].split()]
if which == "config2":
    p, nwin = synth_genome(1, 1_000_000, 25, 25, seed=12345), 2792
else:
    p, nwin = synth_genome(32, 1_562_500, 25, 25, seed=777), 139499
eng = Engine.get(0)
s0 = torch.cuda.Stream()
eng.set_stream(s0.cuda_stream)
dev = eng.upload(p)
streams = [s0.cuda_stream] + [torch.cuda.Stream().cuda_stream for _ in range(5)]
for S, W in combos:
    plans = [eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=fst, scan_wgs_per_cu=W)) for _ in range(S)]
    outs = [torch.zeros((plans[0].nrec, 64), dtype=torch.uint8, device="cuda:0") for _ in range(S)]
    ptrs = [o.data_ptr() for o in outs]
    Plan.run_streams(plans, streams[:S], 4 * S, ptrs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Plan.run_streams(plans, streams[:S], runs, ptrs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / runs
    for k in range(1, S):
        assert torch.equal(outs[k], outs[0])
    for q in plans:
        q.check()
        q.close()
    print(f"{which} {'fst' if fst else 'nofst'} streams {S} wgs/cu {W}: {dt * 1e6:.1f} us per pass, {nwin / dt:.3e} "
          f"windows/s, {(12 * p.n + 64 * nwin) / dt / 1e12:.2f} TB/s (SURVEY 8d bytes)", flush=True)
