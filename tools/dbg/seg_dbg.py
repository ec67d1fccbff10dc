import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "2dsfs-scan_amd"), REPO]
import numpy as np
from sfs2d.vcf import read_vcf
from sfs2d.pack import PackedSNPs
from sfs2d.engine import Engine, ScanConfig
from sfs2d import _lib as L
from oracle import sfs_oracle as O
G = os.path.join(REPO, "tests", "golden")
p = read_vcf(os.path.join(G, "vcf_test.vcf.gz"), os.path.join(G, "popmap_3pop.txt")).to_packed("uv", "bv")
eng = Engine.get(0)

def sub(p, keep):
    keep = np.asarray(keep)
    cs = np.searchsorted(np.nonzero(keep)[0], p.chrom_off)
    return PackedSNPs(p.counts[keep], p.pos[keep], cs.astype(np.int64), p.chrom_names, p.ann_id[keep], p.ann_names)

def check(name, q, ws, n1p=11, n2p=11, fst=False):
    dev = eng.upload(q)
    recs = eng.scan(dev, ScanConfig(n1p=n1p, n2p=n2p, window=ws, fst=fst))
    dev.close()
    got = {(int(r["chrom"]), int(r["wid"])): (int(r["begin"]), int(r["end"])) for r in recs if not r["flags"] & L.W_EMPTY}
    exp = {}
    for c in range(q.nchrom):
        lo, hi = int(q.chrom_off[c]), int(q.chrom_off[c + 1])
        w = (q.pos[lo:hi].astype(np.int64) - 1) // ws
        for u in np.unique(w):
            ii = np.nonzero(w == u)[0]
            exp[(c, int(u))] = (lo + int(ii[0]), lo + int(ii[-1]) + 1)
    miss = sorted(set(exp) - set(got))
    bad = [k for k in exp if k in got and got[k] != exp[k]]
    print(f"{name} ws={ws} fst={fst}: exp {len(exp)} got {len(got)} missing {miss[:12]} wrong {bad[:5]}", flush=True)

for fst in (False, True):
    check("orig", p, 500000, fst=fst)
check("orig", p, 100000)
check("orig", p, 1000000)
check("orig18", p, 500000, 18, 14)
keep = np.ones(p.n, bool); keep[0] = False
check("no-pos5", sub(p, keep), 500000)
dup = np.nonzero(np.diff(p.pos.astype(np.int64)) == 0)[0]
keep = np.ones(p.n, bool); keep[dup] = False
check("no-dup", sub(p, keep), 500000)
q = PackedSNPs(p.counts[:2484], p.pos[:2484], np.array([0, 2484]), p.chrom_names[:1], p.ann_id[:2484], p.ann_names)
check("chrom0", q, 500000)
