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
