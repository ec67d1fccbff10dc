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


@pytest.mark.timeout(600)
def test_config3_genome_wide_background_precomputed():
    """BASELINE config 3's genome-wide-background variant at full size, through the drop-in class as the
    reference script runs it (twoDSFS_class.py:1970-1983 then scan_precomputed_BG, 1161): the whole
    genome's 2D / folded 1D SFS (GPU histograms), normalised in dict order, every 20 kb window scored
    against it.  Window labels and SNP counts for every window from the positions; a 200-window oracle
    sample of the statistics (1e-10 relative) against the oracle's own genome background."""
    import time
    import twoDSFS_class as T
    from sfs2d.synth import synth_genome
    t0 = time.perf_counter()
    log = lambda m: print(f"[config3-genome {time.perf_counter() - t0:6.1f}s] {m}", flush=True)
    p = synth_genome(NCHROM, PER, POP, POP, seed=777)
    log("generated")
    obj = T.LikelihoodInference_jointSFS(None, None, pop1="p1", pop2="p2", pop1_size=POP, pop2_size=POP)
    bg2 = obj.normalize_2d_sfs(obj.calculate_2d_sfs(p))
    bg1 = obj.normalize_1d_sfs(obj.fold_1d_sfs(obj.calculate_1d_sfs(p, "p1", POP, None, None, None)))
    bg1b = obj.normalize_1d_sfs(obj.fold_1d_sfs(obj.calculate_1d_sfs(p, "p2", POP, None, None, None)))
    log("background")
    res = obj.scan_precomputed_BG(p, 20000, bg2, bg1, bg1b)
    log("scanned")
    exp = _expected_windows(p, 20000)
    labels = [f"{p.chrom_names[c]} {1 + w * 20000}-{(w + 1) * 20000}" for c, w in exp[:, :2].tolist()]
    assert list(res) == labels
    assert [r["snp_count"] for r in res.values()] == (exp[:, 3] - exp[:, 2]).tolist()
    ocfg = O.Cfg(POP, POP)
    g = O.genome_backgrounds_normalized(p, ocfg)
    # the oracle's normalised background equals the class's (the same sums in the same order)
    assert np.array_equal(g[0].ravel(), np.array(list(bg2.values()))), "2D background"
    assert np.array_equal(g[1], np.array(list(bg1.values()))) and np.array_equal(g[2], np.array(list(bg1b.values())))
    rng = np.random.default_rng(5)
    sample = np.sort(rng.choice(len(exp), 200, replace=False))
    vals = list(res.values())
    for i in sample:
        q = _win(p, int(exp[i, 2]), int(exp[i, 3]))
        o = O.window_records(q, [(0, 0, q.n)], ocfg, lambda _c: g)[0]
        r = vals[i]
        for f, k in (("T2D", "T2D"), ("T1D_pop1", "T1D_p1"), ("T1D_pop2", "T1D_p2")):
            assert gu.close(r[f], o[k]), (i, f, r[f], o[k])
        assert gu.close(r["new_term_pop1"], None if o["T2D"] is None or o["T1D_p1"] is None else o["T2D"] - o["T1D_p1"])
    log("oracle sample checked")
