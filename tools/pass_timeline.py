#!/usr/bin/env python3
"""Kernel timeline of config-3 passes (for rocprofv3 --kernel-trace): R passes of one plan back to back on
one stream.  usage: rocprofv3 --kernel-trace --output-format csv -d DIR -o tl -- python3 tools/pass_timeline.py [R]
then: python3 tools/pass_timeline.py --read DIR   (start / end of each kernel of the last passes, us)"""
import glob
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 2 and sys.argv[1] == "--read":
    import csv
    f = sorted(glob.glob(os.path.join(sys.argv[2], "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "k_prep" in r["Kernel_Name"] or "k_scan" in r["Kernel_Name"] or "k_bg" in r["Kernel_Name"]]
    last = rows[-12:]
    t0 = int(last[0]["Start_Timestamp"])
    for r in last:
        name = r["Kernel_Name"].split("<")[0].split("(")[0].replace("void ", "").replace("sfs2dk::", "")
        print(f"{name:14s} grid {int(r['Grid_Size_X']):8d}  queue {r.get('Queue_Id', '?'):>3s}  "
              f"start {(int(r['Start_Timestamp']) - t0) / 1e3:8.1f}  end {(int(r['End_Timestamp']) - t0) / 1e3:8.1f}  "
              f"dur {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:7.1f} us")
    sys.exit(0)
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
from sfs2d.engine import Engine, ScanConfig  # noqa: E402
from sfs2d.synth import synth_genome  # noqa: E402
R = int(sys.argv[1]) if len(sys.argv) > 1 else 6
p = synth_genome(32, 1_562_500, 25, 25, seed=777)
eng = Engine.get(0)
dev = eng.upload(p)
pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
pl.run_many(R)
pl.check()
print("ok", flush=True)
