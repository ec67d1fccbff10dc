#!/usr/bin/env python3
"""Diagnostic: bench.py's config-3 overlapped-pass measurement (hbm_stream_roofline) in isolation and
after the bench's own config-2 three-stream loop, to find why it reads slower inside bench.py than
tools/exp_streams_cfg3.py.  usage: python tools/hbm_probe.py [with-loop]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
sys.path.insert(0, REPO)
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch  # noqa: E402

import bench  # noqa: E402
from sfs2d.engine import Engine, Plan, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402

torch.cuda.set_device(0)
eng = Engine.get(0)
scan_s = torch.cuda.Stream(device=0)
torch.cuda.set_stream(scan_s)
eng.set_stream(scan_s.cuda_stream)
if len(sys.argv) > 1 and sys.argv[1] == "with-loop":
    p = synth_genome(1, 1_000_000, 25, 25, seed=12345)
    dev = eng.upload(p)
    plans = [eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True)) for _ in range(3)]
    ss = [scan_s.cuda_stream] + [torch.cuda.Stream(device=0).cuda_stream for _ in range(2)]
    outs = [torch.zeros((plans[0].nrec, 64), dtype=torch.uint8, device="cuda:0") for _ in range(3)]
    Plan.run_streams(plans, ss, 400, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
for rep in range(2):
    r = bench.hbm_stream_roofline(eng)
    print(sys.argv[1:] or ["alone"], rep, "serial %.4f ms" % r["pipeline_ms"],
          "overlapped(Fst) %.4f ms" % r["overlapped"]["pipeline_ms"],
          "t2d_t1d %.4f ms" % r["t2d_t1d_overlapped"]["pipeline_ms"], flush=True)
