"""The C restatement of the oracle (oracle/sfs_oracle_c.c: the bench's CPU baseline) against the
numpy oracle, which tests/test_oracle_golden.py pins to the reference's golden vectors: window
segmentation identical, T2D / T1D within 1e-10 relative (exact zeros within 1e-12 absolute), None
<-> NaN, at any thread count."""
import os
import subprocess

import numpy as np
import pytest

from oracle import sfs_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def oc():
    from oracle import sfs_oracle_c as C
    if not os.path.exists(C.LIB_PATH):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True, capture_output=True)
    return C


def _close(a, b):
    if b is None:
        return np.isnan(a)
    if np.isinf(b):
        return a == b
    return abs(a - b) <= 1e-12 + 1e-10 * abs(b)


@pytest.mark.parametrize("n1p,n2p,ws,threads", [(25, 25, 20000, 1), (25, 25, 20000, 4), (18, 14, 7000, 2),
                                                (3, 2, 500, 3), (50, 50, 100000, 2)])
def test_c_oracle_matches_numpy_oracle(oc, n1p, n2p, ws, threads):
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [4000, 2500, 1], n1p, n2p, seed=n1p * 11 + ws)
    cfg = O.Cfg(n1p, n2p)
    bgs = O.chrom_backgrounds(p, cfg)
    wins = O.bp_windows(p, ws)
    r = oc.scan_bp(p, ws, n1p, n2p, threads)
    assert len(r["b"]) == len(wins)
    for j, (c, start, b, e) in enumerate(wins):
        assert (int(r["chrom"][j]), int(r["start"][j]), int(r["b"][j]), int(r["e"][j])) == (c, start, b, e)
        T2D, f1, f2 = O._stats(p, b, e, cfg, bgs[c])
        t1a, t1b = O.clr1d(f1, bgs[c][1]), O.clr1d(f2, bgs[c][2])
        for got, ref in ((r["T2D"][j], T2D), (r["T1D_p1"][j], t1a), (r["T1D_p2"][j], t1b)):
            assert _close(float(got), None if ref is None else float(ref)), (j, got, ref)


def test_c_oracle_thread_count_independent(oc):
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [30000, 12000], 25, 25, seed=77)
    a = oc.scan_bp(p, 20000, 25, 25, 1)
    b = oc.scan_bp(p, 20000, 25, 25, 4)
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True) if a[k].dtype.kind == "f" else np.array_equal(a[k], b[k])
