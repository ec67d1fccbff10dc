#!/usr/bin/env python3
"""Model of k_scan_w's 2D LDS atomics on the synthetic genome (CPU): how many lanes of a 64-SNP row
hit the same u16-packed 2D word, and how many distinct words share an LDS bank within a 32-lane
group (ds_add_rtn_u32: 2 x 32 lane groups, bank = word mod 32; MI355X_MICROARCH.md §LDS), against
uniformly random words.  The bank-conflict cycles of the scan are mostly this scatter, not a few hot
bins: the hottest bins hold ~3.4% of the SNPs each.
usage: python tools/lds_bank_model.py [n_snp]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "2dsfs-scan_amd"))
from sfs2d.synth import synth_genome  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
p = synth_genome(1, n, 25, 25, seed=12345)
r1, a1, r2, a2 = p.ref1, p.alt1, p.ref2, p.alt2
sw = (a1 + a2) > 50                       # joint fold
x1, x2 = np.where(sw, r1, a1), np.where(sw, r2, a2)
k2 = x1 * 51 + x2                         # 2D key; 0 = bin (0,0), not counted (lane trash word)
h = np.bincount(k2, minlength=51 * 51) / len(k2)
print("bin (0,0):", round(h[0], 4), " hottest counted bins:",
      [(divmod(int(k), 51), round(float(h[k]), 4)) for k in np.argsort(-h)[1:7]])
m = (len(k2) // 64) * 64
K = k2[:m].reshape(-1, 64)
lane = np.arange(64)
trash = 1304 + 4 * 26 * 2 + lane          # per-lane trash words after the wave's histograms
words = np.where(K == 0, trash[None, :], K >> 1)
rng = np.random.default_rng(0)


def group_cost(w):
    """max distinct words on one bank, over the two 32-lane groups (LDS cycles per group)"""
    out = 0
    for g in (w[:32], w[32:]):
        d = {}
        for x in set(g.tolist()):
            d[x % 32] = d.get(x % 32, 0) + 1
        out += max(d.values())
    return out


same = np.mean([np.bincount(r).max() for r in words[:4000]])
cyc = np.mean([group_cost(r) for r in words[:4000]])
rnd = np.mean([group_cost(rng.integers(0, 1304, 64)) for _ in range(4000)])
print(f"lanes on the most-hit word per row: {same:.2f}; LDS cycles per atomic (2 groups, distinct words "
      f"per bank): data {cyc:.2f}, uniformly random words {rnd:.2f}, conflict-free 2")
