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

# gaps between consecutive dispatches (end of one -> start of the next, in start order): the median
# per (previous kernel, next kernel) pair; negative = the two overlapped (other streams)
seq = sorted(rows, key=lambda r: int(r["Start_Timestamp"]))
gaps = collections.defaultdict(list)
for a, b in zip(seq, seq[1:]):
    na = re.sub(r"[<(].*", "", a["Kernel_Name"]).replace("void ", "").replace("sfs2dk::", "")
    nb = re.sub(r"[<(].*", "", b["Kernel_Name"]).replace("void ", "").replace("sfs2dk::", "")
    gaps[(na, nb)].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3)
print("gaps (end of previous dispatch -> start of next), us:")
for (na, nb), v in sorted(gaps.items(), key=lambda kv: -len(kv[1])):
    if len(v) < 8:
        continue
    v.sort()
    print(f"  {na:14s} -> {nb:14s} n={len(v):5d} med={v[len(v)//2]:7.2f}  p10={v[len(v)//10]:7.2f}  p90={v[9*len(v)//10]:7.2f}")
