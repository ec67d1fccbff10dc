"""Seeded synthetic SNP streams (SURVEY.md section 8d generator).

Per chromosome: positions are the cumulative sum of ``1 + floor(Exponential)`` gaps with
mean ``20000/358.5`` bp (the ECB mean SNP density, twoDSFS_class.py:2032 comment), so they
are unique and >= 1.  Ancestral frequency ``f ~ Beta(0.3, 0.3)``; per population
``f_i = clip(f + N(0, 0.05), 0, 1)``; missing alleles ``~ Binomial(2 n_i, 0.02)``;
``alt_i ~ Binomial(2 n_i - miss_i, f_i)``; ``ref_i = 2 n_i - miss_i - alt_i``.
RNG: numpy PCG64 with the given seed, chromosome by chromosome.
"""
from __future__ import annotations

import numpy as np

from .pack import PackedSNPs, pack_counts

MEAN_GAP = 20000.0 / 358.5


def synth_chrom(rng, nsnp: int, n1p: int, n2p: int, miss_rate: float = 0.02, sd: float = 0.05,
                mean_gap: float = MEAN_GAP):
    gaps = 1 + np.floor(rng.exponential(mean_gap - 0.5, size=nsnp)).astype(np.int64)
    pos = np.cumsum(gaps)
    f = rng.beta(0.3, 0.3, size=nsnp)
    f1 = np.clip(f + rng.normal(0.0, sd, size=nsnp), 0.0, 1.0)
    f2 = np.clip(f + rng.normal(0.0, sd, size=nsnp), 0.0, 1.0)
    m1 = rng.binomial(2 * n1p, miss_rate, size=nsnp)
    m2 = rng.binomial(2 * n2p, miss_rate, size=nsnp)
    a1 = rng.binomial(2 * n1p - m1, f1)
    a2 = rng.binomial(2 * n2p - m2, f2)
    r1 = 2 * n1p - m1 - a1
    r2 = 2 * n2p - m2 - a2
    return pos, r1, a1, r2, a2


def synth_genome(nchrom: int, snps_per_chrom, n1p: int, n2p: int, seed: int = 12345,
                 n_ann: int = 1, pop1: str = "p1", pop2: str = "p2", chrom_prefix: str = "chr") -> PackedSNPs:
    """Synthetic genome of ``nchrom`` chromosomes (names sort in Python string order)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    if np.isscalar(snps_per_chrom):
        snps_per_chrom = [int(snps_per_chrom)] * nchrom
    names = [f"{chrom_prefix}{i:04d}" for i in range(nchrom)]
    pos_l, c_l, a_l, offs = [], [], [], [0]
    for c in range(nchrom):
        pos, r1, a1, r2, a2 = synth_chrom(rng, snps_per_chrom[c], n1p, n2p)
        if pos.size and pos[-1] > 0xFFFFFFFF:
            raise ValueError("chromosome too long for uint32 positions")
        pos_l.append(pos.astype(np.uint32))
        c_l.append(pack_counts(r1, a1, r2, a2))
        a_l.append(rng.integers(0, n_ann, size=len(pos)).astype(np.uint16))
        offs.append(offs[-1] + len(pos))
    ann_names = ["intergenic_region", "intron_variant", "missense_variant", "synonymous_variant"][:max(1, n_ann)]
    while len(ann_names) < n_ann:
        ann_names.append(f"ann{len(ann_names)}")
    return PackedSNPs(np.concatenate(c_l) if c_l else np.zeros(0, np.uint32),
                      np.concatenate(pos_l) if pos_l else np.zeros(0, np.uint32),
                      np.array(offs, np.int64), names,
                      np.concatenate(a_l) if a_l else np.zeros(0, np.uint16), ann_names, pop1, pop2)
