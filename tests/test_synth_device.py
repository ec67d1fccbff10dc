"""Device-generated sims replicates (sfs2d_data_synth_sims, BASELINE config 4): bit-exact against
the host twin (sfs2d.synth.sims_host), and the sims scan over the generated data equal to the
oracle's restatement of sims_scan.process_window on the host twin's arrays."""
import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,nwin,nrep", [(50, 40, 6), (5, 25, 3)])
def test_device_equals_host_twin(n, nwin, nrep):
    from sfs2d.engine import Engine
    from sfs2d.synth import miss_table, sims_host, sims_window_counts
    seed, gen = 0x1234567890AB, 3
    wc = sims_window_counts(seed, gen, nrep, nwin)
    mt = miss_table(2 * n)
    eng = Engine.get(0)
    dev = eng.synth_sims(seed, gen, nrep, nwin, 20000, n, n, wc, mt, mt)
    try:
        c, p = dev.read(int(wc.astype(np.int64).sum()))
    finally:
        dev.close()
    host = sims_host(seed, gen, nwin, 20000, n, n, wc, range(nrep), mt, mt)
    assert np.array_equal(c, host.counts)
    assert np.array_equal(p, host.pos)


def test_scan_of_generated_data_vs_oracle():
    import sims_scan as S
    from oracle import sfs_oracle as O
    from sfs2d import _lib as L
    from sfs2d import post
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import miss_table, sims_host, sims_window_counts
    n, nwin, nrep, ws = 5, 30, 4, 20000
    seed, gen = 99, 1
    wc = sims_window_counts(seed, gen, nrep, nwin)
    mt = miss_table(2 * n)
    host = sims_host(seed, gen, nwin, ws, n, n, wc, range(nrep), mt, mt)
    bg2, bg1, bg1b = (S.calculate_2d_sfs(host, "p1", "p2", n, n, 0, 500000, None),
                      S.calculate_1d_sfs(host, "p1", n, 0, 500000, None), S.calculate_1d_sfs(host, "p2", n, 0, 500000, None))
    eng = Engine.get(0)
    dev = eng.synth_sims(seed, gen, nrep, nwin, ws, n, n, wc, mt, mt)
    try:
        cfg = ScanConfig(n1p=n, n2p=n, window=ws, bg_mode=L.BG_SUPPLIED)
        recs = eng.scan(dev, cfg, S._bg_arrays(bg2, bg1, bg1b, n, n))
    finally:
        dev.close()
    o2, o1, o1b = O.sims_backgrounds(host, n, n)
    for r in range(nrep):
        sub = recs[recs["chrom"] == r].copy()
        sub["chrom"] = 0
        q = host.subset_chroms([r])
        got = post.sims_process_window(sub, q, ws, len(sub))
        ref = O.sims_process_window(q, o2, o1, o1b, ws, n, n)
        assert not gu.compare_results(got, ref)


@pytest.mark.parametrize("ws", [20000, 10000])
def test_generator_slots_equal_segmentation(monkeypatch, ws):
    """A fixed-bp plan over generated replicates with the generator's window length takes its slot table
    from the generator's window offsets (k_slots_synth) instead of k_prep's segmentation of the
    positions: the records are byte-equal to the segmentation path's (SFS2D_SEG=prep) and to the binary
    search on the positions (SFS2D_SEG=search, k_slots_search: what real replicate VCFs get), including
    windows without SNPs; another window length (10 kb) takes the search or k_prep either way."""
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import miss_table, sims_window_counts
    n, nwin, nrep = 25, 60, 5
    seed, gen = 4242, 2
    wc = sims_window_counts(seed, gen, nrep, nwin, mean=40.0)
    wc[3] = 0                     # an empty window in replicate 0
    wc[nwin + 7] = 1              # a one-SNP window in replicate 1
    mt = miss_table(2 * n)
    eng = Engine.get(0)
    dev = eng.synth_sims(seed, gen, nrep, nwin, 20000, n, n, wc, mt, mt)
    try:
        h2, u1, u2 = eng.bg_hist(dev, ScanConfig(n1p=n, n2p=n, start_position=0, end_position=500000), -1)
        bg = (h2.reshape(-1).astype(np.float64), u1[: n + 1].astype(np.float64), u2[: n + 1].astype(np.float64))
        cfg = ScanConfig(n1p=n, n2p=n, window=ws, bg_mode=L.BG_SUPPLIED)
        outs = []
        for flag in ("auto", "prep", "search"):
            monkeypatch.setenv("SFS2D_SEG", flag)
            pl = eng.plan(dev, cfg)
            pl.set_background(*bg)
            for _ in range(2):   # the scan clears the slot table after use: a second run rebuilds it
                pl.run()
                pl.check()
            outs.append(pl.read().tobytes())
            pl.close()
    finally:
        dev.close()
    assert outs[0] == outs[1] == outs[2]


@pytest.mark.parametrize("ws", [20000, 3000, 100000])
def test_slot_search_equals_segmentation(monkeypatch, ws):
    """Supplied-background fixed-bp counts plans (scan_chooseChr / scan_precomputed_BG / sims over real
    VCFs) take their slot table from k_slots_search (binary search on the resident positions) instead of
    k_prep's segmentation: byte-equal records on data with empty windows (3 kb), windows of one or two
    SNPs, a one-SNP chromosome, and with Fst (k_prep's sums keep k_prep), on small (k_scan_w) and large
    (k_scan_gw) grids; and the search path against the oracle."""
    from oracle import sfs_oracle as O
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    import golden_util as gu
    eng = Engine.get(0)
    for n in (25, 50):
        p = synth_genome(5, [5000, 1, 3000, 70, 900], n, n, seed=ws + n)
        dev = eng.upload(p)
        cfg_o = O.Cfg(n, n)
        idx = np.arange(p.chrom_off[0], p.chrom_off[1])
        bg = (O.sfs2d(p, idx, cfg_o), O.fold1d(O.sfs1d(p, idx, 1, cfg_o)), O.fold1d(O.sfs1d(p, idx, 2, cfg_o)))
        try:
            for fst in (False, True):
                outs = []
                for flag in ("search", "prep"):
                    monkeypatch.setenv("SFS2D_SEG", flag)
                    pl = eng.plan(dev, ScanConfig(n1p=n, n2p=n, window=ws, bg_mode=L.BG_SUPPLIED, fst=fst))
                    pl.set_background(*bg)
                    for _ in range(2):
                        pl.run()
                        pl.check()
                    outs.append(pl.read())
                    pl.close()
                assert outs[0].tobytes() == outs[1].tobytes()
            recs = outs[0]
            body = recs[(recs["flags"] & L.W_EMPTY) == 0]
            ref = O.window_records(p, O.bp_windows(p, ws), cfg_o, lambda c: bg)
            assert len(body) == len(ref)
            for r, o in zip(body, ref):
                assert int(r["snp_count"]) == o["snp_count"] and int(r["n2"]) == o["N2"]
                for f, g in (("t2d", "T2D"), ("t1d_p1", "T1D_p1"), ("t1d_p2", "T1D_p2")):
                    if o[g] is not None:
                        assert gu.close(float(r[f]), o[g]), (f, float(r[f]), o[g])
        finally:
            dev.close()


@pytest.mark.timeout(600)
def test_config4_shape_generator_slots_vs_oracle():
    """BASELINE config 4's own path at its own shape: pop_size 50 / 50 (101 x 101 grid -> k_scan_gw),
    2,000 windows of 20 kb per replicate, Poisson(358.5) SNPs per window, replicates generated in HBM,
    the slot table from the generator's window offsets (k_slots_synth, the default for this plan), the
    generation's background = every replicate's SNPs at pos <= 500,000 (sims_scan.py:615-617, 1D
    spectra UNFOLDED, quirk Q7).  The device background equals the oracle's on the host twin's arrays
    bit for bit; a sample of windows of three replicates (first / middle / last) equals the oracle's
    restatement of process_window's per-window statistics (sims_scan.py:451-590: T2D, T1D of both
    populations against the unfolded 1D background, snp_count, the inner totals)."""
    from oracle import sfs_oracle as O
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import miss_table, sims_host, sims_window_counts
    n, nwin, nrep, ws = 50, 2000, 20, 20000
    seed, gen = 0xC0F4, 2
    wc = sims_window_counts(seed, gen, nrep, nwin)
    assert wc.min() > 0
    mt = miss_table(2 * n)
    host = sims_host(seed, gen, nwin, ws, n, n, wc, range(nrep), mt, mt)
    o2, o1, o1b = O.sims_backgrounds(host, n, n)
    eng = Engine.get(0)
    dev = eng.synth_sims(seed, gen, nrep, nwin, ws, n, n, wc, mt, mt)
    try:
        h2, u1, u2 = eng.bg_hist(dev, ScanConfig(n1p=n, n2p=n, start_position=0, end_position=500000), -1)
        assert np.array_equal(h2.reshape(o2.shape), o2)
        assert np.array_equal(u1, o1) and np.array_equal(u2, o1b)
        bg = (h2.reshape(-1).astype(np.float64), u1[: n + 1].astype(np.float64), u2[: n + 1].astype(np.float64))
        pl = eng.plan(dev, ScanConfig(n1p=n, n2p=n, window=ws, bg_mode=L.BG_SUPPLIED))
        assert pl.scan_kernel() == "k_scan_gw"
        pl.set_background(*bg)
        pl.run()
        pl.check()
        recs = pl.read()
        pl.close()
    finally:
        dev.close()
    assert len(recs) == nrep * nwin
    assert np.array_equal(recs["chrom"], np.repeat(np.arange(nrep), nwin))
    assert np.array_equal(recs["end"] - recs["begin"], wc.astype(np.uint32))
    cfg = O.Cfg(n, n)
    rng = np.random.default_rng(11)
    checked = 0
    for r in (0, nrep // 2, nrep - 1):
        for w in np.sort(rng.choice(nwin, size=40, replace=False)):
            x = recs[r * nwin + w]
            b, e = int(x["begin"]), int(x["end"])
            idx = np.arange(b, e)
            assert host.chrom_off[r] <= b and e <= host.chrom_off[r + 1]
            g = O.sfs2d(host, idx, cfg)
            f1, f2 = O.fold1d(O.sfs1d(host, idx, 1, cfg)), O.fold1d(O.sfs1d(host, idx, 2, cfg))
            assert int(x["snp_count"]) == e - b
            assert int(x["n2"]) == int(g.ravel()[1:-1].sum())
            assert int(x["n1a"]) == int(f1[1:-1].sum()) and int(x["n1b"]) == int(f2[1:-1].sum())
            for f, want in (("t2d", O.clr2d(g, o2, guards=False)), ("t1d_p1", O.clr1d(f1, o1, guards=False)),
                            ("t1d_p2", O.clr1d(f2, o1b, guards=False))):
                assert gu.close(float(x[f]), want), (r, w, f, float(x[f]), want)
            checked += 1
    assert checked == 120
