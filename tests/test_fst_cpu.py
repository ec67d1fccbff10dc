"""Fst (not in the reference; defined in oracle.window_fst / DESIGN.md): hand-computed known answers."""
import numpy as np

from oracle import sfs_oracle as O
from sfs2d.pack import PackedSNPs, pack_counts


def _packed(rows):
    r1, a1, r2, a2 = (np.array(c) for c in zip(*rows))
    n = len(rows)
    return PackedSNPs(pack_counts(r1, a1, r2, a2), np.arange(1, n + 1) * 10, np.array([0, n]), ["c1"],
                      np.zeros(n, np.uint16))


def test_known_answer_two_snps():
    # SNP A: p1 = 1/4, p2 = 3/4 -> num = 1/4 - 1/16 - 1/16 = 1/8, den = 1/16 + 9/16 = 5/8
    # SNP B: p1 = p2 = 1/2      -> num = -1/12 - 1/12 = -1/6,   den = 1/4 + 1/4 = 1/2
    # Fst = (1/8 - 1/6) / (9/8) = -1/27
    p = _packed([(3, 1, 1, 3), (2, 2, 2, 2)])
    got = O.window_fst(p, np.arange(p.n), O.Cfg(2, 2))
    assert abs(got - (-1.0 / 27.0)) < 1e-15


def test_exclusions():
    cfg = O.Cfg(2, 2)
    # (0,0) after the fold, and a population with a single called allele, are excluded
    p = _packed([(3, 1, 1, 3), (4, 0, 4, 0), (0, 1, 2, 2)])
    assert abs(O.window_fst(p, np.arange(p.n), cfg) - 0.125 / 0.625) < 1e-15
    # nothing qualifies -> None; a fixed difference -> 1 - corrections
    assert O.window_fst(_packed([(4, 0, 4, 0)]), np.arange(1), cfg) is None
    f = O.window_fst(_packed([(4, 0, 0, 4)]), np.arange(1), cfg)
    assert abs(f - 1.0) < 1e-15
    # the joint fold does not change Fst (it is symmetric in the allele labels)
    a = O.window_fst(_packed([(1, 3, 0, 4), (3, 1, 2, 2)]), np.arange(2), cfg)
    b = O.window_fst(_packed([(3, 1, 4, 0), (1, 3, 2, 2)]), np.arange(2), cfg)
    assert abs(a - b) < 1e-15
