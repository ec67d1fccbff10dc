"""Pin the CPU oracle (oracle/sfs_oracle.py) against the reference's own outputs.

Golden vectors come from the reference's unmodified functions (tests/golden/gen_golden.py)
and from the reference's published CSVs (data/ECBstats_*.csv chr1 rows)."""
import math

import numpy as np
import pytest

import golden_util as gu
from oracle import sfs_oracle as O


def oracle_call(p, cfgd, fn, args):
    cfg = O.Cfg(cfgd["n1p"], cfgd["n2p"], cfgd.get("variant_type"), cfgd.get("fold", True),
                cfgd.get("start_position"), cfgd.get("end_position"))
    if fn == "combined_scan":
        return O.combined_scan(p, args[0], cfg)
    if fn == "scan_perChr_bySNPs":
        return O.scan_perChr_bySNPs(p, args[0], cfg)
    if fn == "scan_chooseChr":
        return O.scan_chooseChr(p, args[0], args[1], cfg)
    if fn == "scan_chooseChr_bySNPs":
        return O.scan_chooseChr_bySNPs(p, args[0], args[1], cfg)
    if fn == "scan_precomputed_BG":
        g2, g1a, g1b = O.genome_backgrounds_normalized(p, cfg)
        return O.scan_precomputed_BG(p, args[0], g2, g1a, g1b, cfg)
    if fn in ("T2D_scan", "T1D_scan"):
        _, bg, extra = gu.t12_inputs(p, cfgd, fn, args)
        if fn == "T2D_scan":
            last = None
            if args[-1] is not None:   # the dict's last key, as an index into the scan order
                c, q = args[-1].split("-")
                ci = p.chrom_names.index(c)
                lo, hi = int(p.chrom_off[ci]), int(p.chrom_off[ci + 1])
                last = lo + int(np.searchsorted(p.pos[lo:hi], int(q)))
            n2 = 2 * cfgd["n2p"] + 1
            g = np.array([bg[(k // n2, k % n2)] for k in range(len(bg))]).reshape(-1, n2)
            return O.T2D_scan(p, extra[0], g, cfg, last)
        return O.T1D_scan(p, extra[0], np.array([bg[k] for k in range(len(bg))]), extra[1], extra[2], cfg)
    raise KeyError(fn)


def _calls(golden):
    out = []
    for name in golden.cases():
        for i, c in enumerate(golden.calls(name)):
            if c["fn"] == "sims_process_window":
                continue
            out.append((name, i))
    return out


_G = gu.Golden()


@pytest.mark.parametrize("name,i", _calls(_G), ids=[f"{n}-{i}" for n, i in _calls(_G)])
def test_oracle_matches_reference(golden, name, i):
    call = golden.calls(name)[i]
    p = golden.packed(name)
    ok, out, _ = gu.run_capture(oracle_call, p, golden.cfg(name), call["fn"], call["args"])
    ref = call["out"]
    if not ref["ok"]:
        assert not ok, f"reference raised {ref['error']} but the oracle returned"
        assert type(out).__name__ == ref["error"]
        assert str(out) == ref["message"]
        return
    assert ok, f"oracle raised {out!r}"
    errs = gu.compare_results(out, gu.decode_results(ref["results"]))
    assert not errs, errs[:10]


@pytest.mark.parametrize("tag", ["sims_n10", "sims_n100"])
def test_oracle_sims(golden, tag):
    call = golden.calls(tag)[0]
    rep = golden.packed(tag)
    bgd = golden.packed(f"{tag}_bgdata")
    cfgd = golden.cfg(tag)
    bg2, bg1, bg1b = O.sims_backgrounds(bgd, cfgd["n1p"], cfgd["n2p"])
    gb = golden.npz(f"{tag}_bg.npz")
    assert np.array_equal(bg2, gb["bg2d"]) and np.array_equal(bg1, gb["bg1a"]) and np.array_equal(bg1b, gb["bg1b"])
    out = O.sims_process_window(rep, bg2, bg1, bg1b, 500000, cfgd["n1p"], cfgd["n2p"])
    errs = gu.compare_results(out, gu.decode_results(call["out"]["results"]))
    assert not errs, errs[:10]


def test_oracle_chr1_background_bitexact(golden):
    p = golden.packed("chr1")
    cfg = O.Cfg(18, 14)
    bg2, bg1a, bg1b = O.chrom_backgrounds(p, cfg)[0]
    g = golden.npz("chr1_bg.npz")
    assert np.array_equal(bg2, g["bg2d"])
    assert np.array_equal(bg1a, g["bg1a"])
    assert np.array_equal(bg1b, g["bg1b"])


@pytest.mark.parametrize("fname,ws", [("ECBstats_500kb.csv", 500000)])
def test_oracle_vs_published_csv(golden, fname, ws):
    """The published CSVs were written by R with 15 significant digits."""
    pub = golden.published()[fname]
    p = golden.packed("chr1")
    out = O.combined_scan(p, ws, O.Cfg(18, 14))
    rows = {(int(r["window_start"]), int(r["window_end"])): r for r in pub}
    assert len(rows) == len(out)
    for k, d in out.items():
        s, e = k.split(" ")[1].split("-")
        r = rows[(int(s), int(e))]
        assert int(r["snp_count"]) == d["snp_count"]
        for f_ref, f in [("T2D", "T2D"), ("T1D_p1", "T1D_pop1"), ("T1D_p2", "T1D_pop2"),
                         ("new_term_p1", "new_term_pop1"), ("new_term_p2", "new_term_pop2"), ("T2D_diff", "T2D_diff")]:
            assert math.isclose(float(r[f_ref]), d[f], rel_tol=1e-12), (k, f)
