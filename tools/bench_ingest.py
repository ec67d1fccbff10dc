#!/usr/bin/env python3
"""Time the native VCF ingest (sfs2d.vcf) against the Python restatement of make_data_dict_vcf.

usage: python tools/bench_ingest.py [n_records] [threads]
Writes a synthetic BGZF VCF (32 samples, 18 uv + 14 bv like the reference's popmap) to /tmp.
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))
from gen_golden_vcf import bgzf_bytes  # noqa: E402
from sfs2d import vcf as V  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
T = int(sys.argv[2]) if len(sys.argv) > 2 else 0
path, pm = f"/tmp/bench_{n}.vcf.gz", "/tmp/bench_popmap.txt"
samples = [f"S{i}" for i in range(32)]
with open(pm, "w") as fh:
    fh.write("".join(f"{s}\t{'uv' if i < 18 else 'bv'}\n" for i, s in enumerate(samples)))
if not os.path.exists(path):
    rng = np.random.default_rng(1)
    gts = np.array(["0/0", "0/1", "1/1", "./.", "1/0"])
    g = gts[rng.choice(5, size=(n, 32), p=[0.5, 0.2, 0.15, 0.05, 0.1])]
    pos = np.cumsum(rng.integers(1, 110, n))
    rows = ["\t".join(["chr1", str(p), ".", "A", "G", ".", "PASS", "PR", "GT"] + list(r)) for p, r in zip(pos, g)]
    head = "##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples) + "\n"
    with open(path, "wb") as fh:
        fh.write(bgzf_bytes((head + "\n".join(rows) + "\n").encode()))
t0 = time.perf_counter()
tab = V.read_vcf(path, pm, nthreads=T)
t1 = time.perf_counter()
pk = tab.to_packed("uv", "bv")
t2 = time.perf_counter()
print(f"native: {n} records, read {t1 - t0:.3f} s ({n / (t1 - t0):.3g} rec/s; {tab.stats}), to_packed {t2 - t1:.3f} s")
if n <= 200_000:
    from oracle import vcf_oracle
    t0 = time.perf_counter()
    d = vcf_oracle.make_data_dict_vcf(path, pm)
    t1 = time.perf_counter()
    print(f"python restatement: {t1 - t0:.3f} s ({n / (t1 - t0):.3g} rec/s)")
