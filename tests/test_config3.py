"""BASELINE config 3 at full size on one GPU: the 5e7-SNP, 32-chromosome synthetic genome (SURVEY 8d
generator), 20 kb + 500 kb windows from ONE pass (a base plan and an attached plan, sfs2d_plan_attach),
per-chromosome backgrounds, Hudson Fst.  Size-independent properties over every window, bit-exact
backgrounds and an oracle sample (1e-10 relative) for the statistics."""
import numpy as np
import pytest

import golden_util as gu
from oracle import sfs_oracle as O

pytestmark = pytest.mark.gpu

NCHROM, PER, POP = 32, 1_562_500, 25


def _expected_windows(p, ws):
    """(chrom, window id, begin, end) of every non-empty fixed-bp window, from the positions."""
    out = []
    for c in range(p.nchrom):
        lo, hi = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
        w = (np.maximum(p.pos[lo:hi].astype(np.int64), 1) - 1) // ws
        cut = np.nonzero(np.diff(w))[0] + 1
        b = np.concatenate([[0], cut]) + lo
        e = np.concatenate([cut, [hi - lo]]) + lo
        out.append(np.stack([np.full(len(b), c), w[b - lo], b, e], axis=1))
    return np.concatenate(out)


def _win(p, b, e):
    from sfs2d.pack import PackedSNPs
    return PackedSNPs(p.counts[b:e], p.pos[b:e], np.array([0, e - b]), ["w"], p.ann_id[b:e], list(p.ann_names),
                      p.pop1, p.pop2)


@pytest.mark.timeout(600)
def test_config3_full_size_20kb_500kb_one_pass():
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    import time
    t0 = time.perf_counter()
    log = lambda m: print(f"[config3 {time.perf_counter() - t0:6.1f}s] {m}", flush=True)
    p = synth_genome(NCHROM, PER, POP, POP, seed=777)   # the stream bench.py's roofline_hbm times
    assert p.n == 50_000_000
    log("generated")
    eng = Engine.get(0)
    dev = eng.upload(p)
    base = eng.plan(dev, ScanConfig(n1p=POP, n2p=POP, window=20000, fst=True))
    big = base.attach(ScanConfig(n1p=POP, n2p=POP, window=500000, fst=True))
    base.run()
    base.check()
    big.check()
    tabs = {20000: (base.read(), base.read_fst()), 500000: (big.read(), big.read_fst())}
    log("scanned")
    # per-chromosome backgrounds: inner 2D sums for every chromosome, bit-exact tables for three
    ocfg = O.Cfg(POP, POP)
    pick = [0, 13, 31]
    bgo = {}
    inner = np.zeros(NCHROM, np.int64)
    for c in range(NCHROM):
        h2, u1, u2 = eng.bg_hist(dev, ScanConfig(n1p=POP, n2p=POP), c)
        inner[c] = int(np.asarray(h2).ravel()[1:-1].sum())
        if c in pick:
            idx = np.arange(p.chrom_off[c], p.chrom_off[c + 1])
            o2, o1, o1b = O.sfs2d(p, idx, ocfg), O.sfs1d(p, idx, 1, ocfg), O.sfs1d(p, idx, 2, ocfg)
            assert np.array_equal(np.asarray(h2), o2) and np.array_equal(u1, o1) and np.array_equal(u2, o1b), c
            bgo[c] = (o2, O.fold1d(o1), O.fold1d(o1b))
    log("backgrounds")
    rng = np.random.default_rng(3)
    for ws, (recs, fst) in tabs.items():
        live = (recs["flags"] & L.W_EMPTY) == 0
        body = recs[live]
        exp = _expected_windows(p, ws)
        # the windows partition the stream exactly: same windows, same SNP ranges, every SNP once
        assert len(body) == len(exp), ws
        got = np.stack([body["chrom"], body["wid"], body["begin"], body["end"]], axis=1).astype(np.int64)
        assert np.array_equal(got, exp), ws
        assert int(body["snp_count"].sum()) == p.n
        # each chromosome's window 2D counts add up to its background's inner sum
        per = np.bincount(body["chrom"].astype(np.int64), weights=body["n2"].astype(np.float64), minlength=NCHROM)
        assert np.array_equal(per.astype(np.int64), inner), ws
        # oracle sample: 200 windows of the three chromosomes with oracle backgrounds
        cand = np.nonzero(np.isin(exp[:, 0], pick))[0]
        sample = np.sort(rng.choice(cand, 200, replace=False))
        # (the oracle reads whole-array fields of its input: one small packed set per window)
        ref = [O.window_records(_win(p, int(exp[i, 2]), int(exp[i, 3])), [(0, 0, int(exp[i, 3] - exp[i, 2]))], ocfg,
                                lambda _c, c=int(exp[i, 0]): bgo[c])[0] for i in sample]
        for i, o in zip(sample, ref):
            r = body[i]
            for f, g in (("snp_count", "snp_count"), ("n2", "N2"), ("n1a", "N1a"), ("n1b", "N1b")):
                assert int(r[f]) == o[g], (ws, i, f)
            for f, g in (("t2d", "T2D"), ("t1d_p1", "T1D_p1"), ("t1d_p2", "T1D_p2")):
                assert gu.close(float(r[f]), o[g]), (ws, i, f, float(r[f]), o[g])
        # Fst (this framework's Hudson estimator; parity vs its own oracle restatement)
        fl = fst[: len(live)][live[: len(fst)]]
        for i in sample[::4]:
            q = _win(p, int(exp[i, 2]), int(exp[i, 3]))
            want = O.window_fst(q, np.arange(q.n), ocfg)
            a = float(fl[i])
            assert (np.isnan(a) if want is None else abs(a - want) <= 1e-12 + 1e-10 * abs(want)), (ws, i)
        log(f"{ws} bp windows checked")
    base.close()
    dev.close()
