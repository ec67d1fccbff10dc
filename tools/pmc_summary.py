#!/usr/bin/env python3
"""Average PMC counters per (kernel, grid) over the passes written by tools/pmc_k3.sh, plus HBM bytes
per launch corrected as MI355X_MICROARCH.md prescribes: FETCH_SIZE (KiB) reads half the bytes of
wide streaming reads on gfx950 -> x2; WRITE_SIZE (KiB) exact.  Writes a CSV to stdout.
usage: python tools/pmc_summary.py gpurun_out/<tag>/pmc_<config> [--json source-label]
(--json: {"source": label, "kernels": [{kernel, grid, read_bytes, write_bytes}]}, what bench.py reads
from profiles/pmc_bench.json for roofline.traffic)"""
import json
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
if len(sys.argv) > 3 and sys.argv[2] == "--json":
    ks = []
    for (name, grid), v in agg.items():
        avg = {c: sum(x) / len(x) for c, x in v.items()}
        ks.append({"kernel": name, "grid": int(grid), "launches": len(v.get("FETCH_SIZE", [])),
                   "read_bytes": 2 * avg.get("FETCH_SIZE", float("nan")) * 1024,
                   "write_bytes": avg.get("WRITE_SIZE", float("nan")) * 1024})
    json.dump({"source": sys.argv[3], "kernels": ks}, sys.stdout, indent=1)
    sys.exit(0)
w = csv.writer(sys.stdout)
w.writerow(["kernel", "grid"] + cols + ["hbm_read_bytes_x2", "hbm_write_bytes"])
for (name, grid), v in agg.items():
    avg = {c: sum(x) / len(x) for c, x in v.items()}
    rd = 2 * avg.get("FETCH_SIZE", float("nan")) * 1024
    wr = avg.get("WRITE_SIZE", float("nan")) * 1024
    w.writerow([name, grid] + [f"{avg.get(c, float('nan')):.6g}" for c in cols] + [f"{rd:.6g}", f"{wr:.6g}"])
