import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "2dsfs-scan_amd"), REPO]
import numpy as np
import twoDSFS_class as T
from sfs2d.vcf import read_vcf
from oracle import sfs_oracle as O
G = os.path.join(REPO, "tests", "golden")
p = read_vcf(os.path.join(G, "vcf_test.vcf.gz"), os.path.join(G, "popmap_3pop.txt")).to_packed("uv", "bv")
obj = T.LikelihoodInference_jointSFS(None, None, pop1_size=11, pop2_size=11)
for ws in (500000, 1000000):
    r = obj.combined_scan(p, ws)
    o = O.combined_scan(p, ws, O.Cfg(11, 11))
    print(ws, len(r), len(o), list(r)[:3], list(r)[-3:])
from sfs2d.engine import Engine, ScanConfig
from sfs2d import _lib as L
eng = Engine.get(0)
dev = eng.upload(p)
recs = eng.scan(dev, ScanConfig(n1p=11, n2p=11, window=500000, prev_extra=True))
print(len(recs), recs[["chrom", "wid", "begin", "end", "snp_count", "n2", "flags"]][:45])
