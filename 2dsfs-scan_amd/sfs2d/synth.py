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


# ----------------------------------------------------------------------------- sims (config 4)
# BASELINE config 4: replicate data sets of n_windows fixed windows with Poisson(358.5) SNPs each,
# generated in HBM by the library (sfs2d_data_synth_sims, kernel k_synth_sims); the functions below
# are the host side: the per-window SNP counts and missing-allele tables (inputs of both sides) and
# ``sims_host``, the bit-exact host twin of the device generator (test infrastructure for parity).

SIMS_MEAN = 358.5
SIMS_MISS = 0.02


def sims_window_counts(seed: int, generation: int, n_rep: int, n_win: int, mean: float = SIMS_MEAN) -> np.ndarray:
    """SNPs per window, uint16 [n_rep * n_win] (PCG64 keyed by (seed, generation))."""
    rng = np.random.Generator(np.random.PCG64([seed, generation]))
    return np.minimum(rng.poisson(mean, size=n_rep * n_win), 65535).astype(np.uint16)


def miss_table(n: int, rate: float = SIMS_MISS) -> np.ndarray:
    """u32 inverse-CDF thresholds of Binomial(n, rate): k missing alleles for the smallest k with
    x < table[k] (x a uniform u32); the last entry is 0xffffffff."""
    from math import comb
    cdf, acc = [], 0.0
    for k in range(n + 1):
        acc += comb(n, k) * rate ** k * (1.0 - rate) ** (n - k)
        cdf.append(acc)
    t = np.minimum(np.floor(np.array(cdf) * 4294967296.0), 4294967295.0).astype(np.uint64)
    t[-1] = 0xFFFFFFFF
    return t.astype(np.uint32)


_M = np.uint64(0xFFFFFFFF)


def _philox(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 on uint64 arrays holding 32-bit lanes (the device's philox4x32)."""
    c0, c1, c2, c3 = (np.asarray(x, np.uint64) for x in (c0, c1, c2, c3))
    k0 = np.uint64(k0)
    k1 = np.uint64(k1)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        h0, l0, h1, l1 = p0 >> np.uint64(32), p0 & _M, p1 >> np.uint64(32), p1 & _M
        c0, c1, c2, c3 = h1 ^ c1 ^ k0, l1, h0 ^ c3 ^ k1, l0
        k0 = (k0 + np.uint64(0x9E3779B9)) & _M
        k1 = (k1 + np.uint64(0xBB67AE85)) & _M
    return c0, c1, c2, c3


def _u01(x):
    return (x.astype(np.float64) + 0.5) * 2.3283064365386963e-10


def _alt(f, m, z4):
    z = (((_u01(z4[0]) + _u01(z4[1])) + (_u01(z4[2]) + _u01(z4[3]))) - 2.0) * 1.7320508075688772
    mf = m.astype(np.float64) * f
    sd = np.sqrt(mf * (1.0 - f))
    x = np.floor((mf + sd * z) + 0.5)
    return np.where(x <= 0.0, 0, np.where(x >= m, m, np.clip(x, 0, None))).astype(np.int64)


def sims_host(seed: int, generation: int, n_win: int, window_bp: int, n1p: int, n2p: int,
              win_counts: np.ndarray, replicates, mt1=None, mt2=None) -> PackedSNPs:
    """The device generator's output for the given replicate indices, computed on the host."""
    mt1 = miss_table(2 * n1p) if mt1 is None else mt1
    mt2 = miss_table(2 * n2p) if mt2 is None else mt2
    woff = np.concatenate([[0], np.cumsum(win_counts.astype(np.uint64))]).astype(np.uint64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    cs, ps, offs, names = [], [], [0], []
    for r in replicates:
        w0 = r * n_win
        kk = win_counts[w0:w0 + n_win].astype(np.int64)
        wl = np.repeat(np.arange(n_win, dtype=np.int64), kk)
        j = np.arange(int(kk.sum()), dtype=np.int64) - np.repeat(np.cumsum(kk) - kk, kk)
        g = woff[w0] + np.arange(int(kk.sum()), dtype=np.uint64)
        lo, hi = g & _M, g >> np.uint64(32)
        a = _philox(lo, hi, 0, generation, k0, k1)
        b = _philox(lo, hi, 1, generation, k0, k1)
        z1 = _philox(lo, hi, 2, generation, k0, k1)
        z2 = _philox(lo, hi, 3, generation, k0, k1)
        u = _u01(a[0])
        u3 = (u * u) * u
        f = np.where((b[3] & np.uint64(1)) != 0, u3, 1.0 - u3)
        f1 = np.minimum(1.0, np.maximum(0.0, f + 0.1 * (_u01(a[2]) - 0.5)))
        f2 = np.minimum(1.0, np.maximum(0.0, f + 0.1 * (_u01(a[3]) - 0.5)))
        miss1 = np.minimum(np.searchsorted(mt1, b[0].astype(np.uint32), side="right"), len(mt1) - 1)
        miss2 = np.minimum(np.searchsorted(mt2, b[1].astype(np.uint32), side="right"), len(mt2) - 1)
        m1, m2 = 2 * n1p - miss1, 2 * n2p - miss2
        a1, a2 = _alt(f1, m1, z1), _alt(f2, m2, z2)
        t = (j.astype(np.float64) + _u01(b[2])) * float(window_bp)
        pos = wl * window_bp + 1 + np.floor(t / np.repeat(kk, kk).astype(np.float64)).astype(np.int64)
        cs.append(pack_counts(m1 - a1, a1, m2 - a2, a2))
        ps.append(pos.astype(np.uint32))
        offs.append(offs[-1] + len(pos))
        names.append(f"rep{r:05d}")
    return PackedSNPs(np.concatenate(cs), np.concatenate(ps), np.array(offs, np.int64), names,
                      np.zeros(offs[-1], np.uint16), ["intergenic_region"], "p1", "p2")
