"""Multi-resolution scans (sfs2d_plan_attach / LikelihoodInference_jointSFS.multi_scan): every window
size from one k_prep pass must give exactly what the single-size drivers give, and the chr1 case the
reference's own outputs (tests/golden, twoDSFS_class.py:787-991, 1422-1541)."""
import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu

_G = gu.Golden()


def _obj(n1p, n2p, pop1="uv", pop2="bv"):
    import twoDSFS_class as T
    return T.LikelihoodInference_jointSFS(None, None, pop1=pop1, pop2=pop2, pop1_size=n1p, pop2_size=n2p)


def _same(a, b):
    assert list(a) == list(b)
    for k in a:
        assert a[k] == b[k] or all(gu.close(a[k][f], b[k][f]) for f in a[k]), k


def test_chr1_against_reference():
    p = _G.packed("chr1")
    cfg = _G.cfg("chr1")
    obj = _obj(cfg["n1p"], cfg["n2p"], cfg["pop1"], cfg["pop2"])
    res = obj.multi_scan(p, [500000, 20000], [500])
    calls = {(c["fn"], tuple(c["args"])): c for c in _G.calls("chr1")}
    for key, got in ((("combined_scan", (20000,)), res[20000]), (("combined_scan", (500000,)), res[500000]),
                     (("scan_perChr_bySNPs", (500,)), res["500snps"])):
        ref = gu.decode_results(calls[key]["out"]["results"])
        errs = gu.compare_results(got, ref)
        assert not errs, (key, errs[:5])


@pytest.mark.parametrize("seed", [1, 2])
def test_matches_single_plans(seed):
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [40000, 25000, 9000], 25, 25, seed=seed)
    obj = _obj(25, 25)
    res = obj.multi_scan(p, [20000, 100000, 60000, 30000, 500000], [500, 300], fst=True)
    for ws in (20000, 30000, 60000, 100000, 500000):
        _same(res[ws], obj.combined_scan(p, ws))
        single = obj.window_fst(p, window_size=ws)
        assert list(res["fst"][ws]) == list(single)
        for k, v in single.items():
            w = res["fst"][ws][k]
            assert (v is None and w is None) or abs(w - v) <= 1e-9 * max(1.0, abs(v)), (ws, k, w, v)
    for S in (500, 300):
        _same(res[f"{S}snps"], obj.scan_perChr_bySNPs(p, S))


def test_large_grid_matches_single_plans():
    """Attached plans on the large-grid path (101 x 101: k_scan_gw with its own exact-path slots)."""
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [30000, 12000, 5000], 50, 50, seed=9)
    obj = _obj(50, 50)
    res = obj.multi_scan(p, [20000, 100000, 500000], [400], fst=True)
    for ws in (20000, 100000, 500000):
        _same(res[ws], obj.combined_scan(p, ws))
        single = obj.window_fst(p, window_size=ws)
        assert list(res["fst"][ws]) == list(single)
        for k, v in single.items():
            w = res["fst"][ws][k]
            assert (v is None and w is None) or abs(w - v) <= 1e-9 * max(1.0, abs(v)), (ws, k, w, v)
    _same(res["400snps"], obj.scan_perChr_bySNPs(p, 400))


def test_repeated_runs_identical():
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [30000, 12000], 25, 25, seed=7)
    eng = Engine.get(0)
    dev = eng.upload(p)
    try:
        base = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, prev_extra=True, fst=True))
        a1 = base.attach(ScanConfig(n1p=25, n2p=25, window=500000, prev_extra=True, fst=True))
        a2 = base.attach(ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=500))
        with pytest.raises(Exception):
            a1.run()   # attached plans run with their base
        outs = []
        for _ in range(3):
            base.run()
            base.check()
            outs.append([pl.read().tobytes() for pl in (base, a1, a2)] + [a1.read_fst().tobytes()])
        assert outs[0] == outs[1] == outs[2]
        # Fst on SNP-count windows: a counts plan's scan sums its own Fst (fst_scan)
        a3 = base.attach(ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=300, fst=True))
        base.run()
        base.check()
        f3, r3 = a3.read_fst(), a3.read()
        from oracle import sfs_oracle as O
        wins = O.snp_windows(p, 300)[0]
        assert len(wins) == len(r3) and list(r3["begin"]) == [w[3] for w in wins]
        for (c, sp, ep, b, e), f in zip(wins, f3):
            v = O.window_fst(p, np.arange(b, e), O.Cfg(25, 25))
            assert (v is None and np.isnan(f)) or abs(f - v) <= 1e-10 * max(1.0, abs(v)), (b, f, v)
        with pytest.raises(Exception):   # a different grid
            base.attach(ScanConfig(n1p=20, n2p=25, window=500000))
        base.close()
        assert not a1.h and not a2.h
    finally:
        dev.close()


def test_attach_fst_without_fst_scan(monkeypatch):
    """SFS2D_FST_SCAN=0 (Fst from k_prep's sums or k_fst_win): attached Fst needs fixed-bp windows."""
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    monkeypatch.setenv("SFS2D_FST_SCAN", "0")
    p = synth_genome(2, [30000, 12000], 25, 25, seed=7)
    eng = Engine.get(0)
    dev = eng.upload(p)
    try:
        base = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, prev_extra=True, fst=True))
        with pytest.raises(Exception):
            base.attach(ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=300, fst=True))
        a = base.attach(ScanConfig(n1p=25, n2p=25, window=100000, fst=True))
        base.run()
        base.check()
        assert np.isfinite(a.read_fst()).any()
        base.close()
    finally:
        dev.close()
