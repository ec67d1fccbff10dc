#!/usr/bin/env python3
"""Copy the chr1 (NC_087088_1) rows of the reference's pixy Fst tables (data files
pixy_data/fst_20kb.csv, fst_500kb.csv) into tests/golden/ -- inputs of the FST-join test (the
published data/ECBstats_*.csv FST column is pixy's avg_wc_fst joined in ECBstats_plots.R:16-41).
Run: python tests/golden/gen_pixy_fixture.py  (build container only)"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))
for res in ("20kb", "500kb"):
    with open(f"/root/reference/pixy_data/fst_{res}.csv", encoding="utf-8-sig") as fh:
        lines = fh.read().splitlines()
    keep = [lines[0]] + [ln for ln in lines[1:] if ln.split(",")[2] == "NC_087088_1"]
    with open(os.path.join(HERE, f"pixy_fst_chr1_{res}.csv"), "w") as fh:
        fh.write("\n".join(keep) + "\n")
    print(res, len(keep) - 1, "rows")
