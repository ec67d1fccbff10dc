#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: mean/min duration per (kernel, grid size).
usage: python tools/ktrace.py <..._kernel_trace.csv>"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("sfs2dk::", "")
    grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
    agg[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{name:40s} grid={grid:9d} n={len(v):4d} mean={sum(v)/len(v):9.2f}us  min={v[0]:8.2f}  med={v[len(v)//2]:8.2f}")
