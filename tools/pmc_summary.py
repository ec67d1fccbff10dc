#!/usr/bin/env python3
"""Average PMC counters per (kernel, grid) over the passes written by tools/pmc_k3.sh, plus HBM bytes
per launch corrected as MI355X_MICROARCH.md prescribes: FETCH_SIZE (KiB) reads half the bytes of
wide streaming reads on gfx950 -> x2; WRITE_SIZE (KiB) exact.  Writes a CSV to stdout.
usage: python tools/pmc_summary.py gpurun_out/<tag>/pmc_<config>"""
import collections
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "pmc_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sfs2dk::", "")
        if "rocclr" in name or "init_lnx" in name:
            continue
        grid = r.get("Grid_Size") or r.get("Grid_Size_X")
        agg[(name, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))
cols = sorted({c for v in agg.values() for c in v})
w = csv.writer(sys.stdout)
w.writerow(["kernel", "grid"] + cols + ["hbm_read_bytes_x2", "hbm_write_bytes"])
for (name, grid), v in agg.items():
    avg = {c: sum(x) / len(x) for c, x in v.items()}
    rd = 2 * avg.get("FETCH_SIZE", float("nan")) * 1024
    wr = avg.get("WRITE_SIZE", float("nan")) * 1024
    w.writerow([name, grid] + [f"{avg.get(c, float('nan')):.6g}" for c in cols] + [f"{rd:.6g}", f"{wr:.6g}"])
