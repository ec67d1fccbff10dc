"""The decomposition k_prep's joint-histogram path (JNT, csrc/sfs2d_kernels.hpp prep_tile) relies on,
checked in numpy against the oracle's own background spectra (oracle.sfs2d / sfs1d, twoDSFS_class.py
140-232 and 398-444): count every SNP once at its unfolded alt-count key (a1, a2) and a folded SNP
(a1 + a2 > n1p + n2p) once more at its (r1, r2) key; then

* both unfolded 1D spectra are the joint grid's margins (bins a >= 1),
* the 2D background is the folded SNPs' (r1, r2) grid plus the joint grid's bins with
  a1 + a2 <= n1p + n2p (the unfolded SNPs' keys), bin (0, 0) excluded,

for folded and unfolded plans, with missing calls and with over-called SNPs (r + a > 2 pop_size)."""
import numpy as np
import pytest

from oracle import sfs_oracle as O


def _joint_decomposition(p, cfg):
    n1, n2 = 2 * cfg.n1p, 2 * cfg.n2p
    r1, a1 = p.counts & 0xFF, (p.counts >> 8) & 0xFF
    r2, a2 = (p.counts >> 16) & 0xFF, p.counts >> 24
    r1, a1, r2, a2 = (x.astype(np.int64) for x in (r1, a1, r2, a2))
    thr = cfg.n1p + cfg.n2p if cfg.fold else np.iinfo(np.int64).max
    sw = (a1 + a2) > thr
    J = np.bincount(a1 * (n2 + 1) + a2, minlength=(n1 + 1) * (n2 + 1)).reshape(n1 + 1, n2 + 1)
    kr = (r1 * (n2 + 1) + r2)[sw]
    H = np.bincount(kr, minlength=(n1 + 1) * (n2 + 1)).reshape(n1 + 1, n2 + 1)
    x1, x2 = np.meshgrid(np.arange(n1 + 1), np.arange(n2 + 1), indexing="ij")
    H2 = H + np.where(x1 + x2 <= thr, J, 0)
    H2[0, 0] = 0
    u1 = J.sum(axis=1)
    u2 = J.sum(axis=0)
    u1[0] = 0
    u2[0] = 0
    return H2, u1, u2


@pytest.mark.parametrize("n1p,n2p,fold,over", [(25, 25, True, False), (25, 25, False, False), (18, 14, True, False),
                                              (3, 2, True, False), (25, 25, True, True), (18, 14, False, True)])
def test_joint_histogram_decomposition(n1p, n2p, fold, over):
    from sfs2d.pack import PackedSNPs, pack_counts
    from sfs2d.synth import synth_genome
    p = synth_genome(1, 40000, n1p, n2p, seed=n1p * 31 + n2p + 7 * fold + over)
    if over:   # over-called SNPs that stay unfolded and inside the grid (the reference counts them)
        r1, a1 = p.counts & 0xFF, (p.counts >> 8) & 0xFF
        r2, a2 = (p.counts >> 16) & 0xFF, p.counts >> 24
        pick = (np.random.default_rng(1).random(p.n) < 0.01) & (a1 + a2 <= n1p + n2p)
        p = PackedSNPs(pack_counts(np.where(pick, r1 + 5, r1), a1, r2, a2), p.pos, p.chrom_off, p.chrom_names,
                       p.ann_id, p.ann_names)
    cfg = O.Cfg(n1p, n2p, fold=fold)
    idx = np.arange(p.n)
    H2, u1, u2 = _joint_decomposition(p, cfg)
    assert np.array_equal(H2, O.sfs2d(p, idx, cfg))
    assert np.array_equal(u1, O.sfs1d(p, idx, 1, cfg))
    assert np.array_equal(u2, O.sfs1d(p, idx, 2, cfg))
