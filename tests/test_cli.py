"""CLI (python -m sfs2d): VCF + popmap -> per-window CSV, and the pixy FST join.

CPU: the CSV writer and the FST join against the published data/ECBstats_*.csv chr1 rows (the
FST column there is pixy's avg_wc_fst joined by ECBstats_plots.R:16-41; the window labels come
from the reference's own combined_scan output in the chr1 golden vectors).
GPU: the full command on the golden test VCF against the oracle's combined_scan / bySNPs drivers.
"""
import csv
import os

import numpy as np
import pytest

from golden_util import GOLD, close, decode_results

import twoDSFS_class as T
from sfs2d import cli


def _read(path):
    with open(path, newline="") as fh:
        return list(csv.DictReader(fh))


@pytest.mark.parametrize("res,ws,call", [("20kb", 20000, 0), ("500kb", 500000, 1)])
def test_pixy_join_matches_published(golden, tmp_path, res, ws, call):
    stats = decode_results(golden.calls("chr1")[call]["out"]["results"])
    pixy = cli.read_pixy_fst(os.path.join(GOLD, f"pixy_fst_chr1_{res}.csv"))
    out = str(tmp_path / "o.csv")
    cli.write_csv(out, stats, {"NC_087088.1": "1"}, pixy=pixy)
    rows = _read(out)
    assert list(rows[0].keys()) == T.col_names + ["FST"]
    pub = {(r["window_start"], r["window_end"]): r for r in golden.published()[f"ECBstats_{res}.csv"]}
    n = 0
    for r in rows:
        p = pub.get((r["window_start"], r["window_end"]))
        if p is None:
            continue
        n += 1
        assert r["chromosome"] == p["chromosome"] == "1"
        if p["FST"] in ("", "NA"):
            assert r["FST"] == ""
        else:
            assert abs(float(r["FST"]) - float(p["FST"])) <= 1e-12 * max(1.0, abs(float(p["FST"])))
        for f in ("snp_count",):
            assert r[f] == p[f]
        for f in ("T2D", "T1D_p1", "T1D_p2"):
            if p[f] not in ("", "NA"):
                assert close(float(r[f]), float(p[f]), rel=1e-12)
    assert n == len(pub) and n > 30


def test_write_csv_matches_save_csv_stats(golden, tmp_path):
    stats = decode_results(golden.calls("chr1")[1]["out"]["results"])
    a, b = str(tmp_path / "a.csv"), str(tmp_path / "b.csv")
    saved = dict(T.chr_ids)
    T.chr_ids.clear()
    T.chr_ids["NC_087088.1"] = "1"
    try:
        T.save_csv_stats(stats, a)
    finally:
        T.chr_ids.clear()
        T.chr_ids.update(saved)
    cli.write_csv(b, stats, {"NC_087088.1": "1"})
    assert open(a).read() == open(b).read()
    assert open(a).read() == open(os.path.join(GOLD, "chr1_500kb_save_csv_stats.csv")).read()


@pytest.mark.gpu
def test_cli_end_to_end(tmp_path):
    from oracle import sfs_oracle as O
    from sfs2d.vcf import read_vcf
    vcf, pm = os.path.join(GOLD, "vcf_test.vcf.gz"), os.path.join(GOLD, "popmap_3pop.txt")
    prefix = str(tmp_path / "run")
    base = [vcf, pm, "--pop1", "uv", "--pop2", "bv", "--pop1-size", "11", "--pop2-size", "11", "--fst",
            "--out-prefix", prefix]
    # the LD-pruned data leaves the first 20 kb window without a T1D: the reference's combined_scan
    # raises UnboundLocalError there (quirk Q6), and so do the oracle and this CLI
    p = read_vcf(vcf, pm).to_packed("uv", "bv")
    cfg = O.Cfg(11, 11)
    with pytest.raises(UnboundLocalError):
        O.combined_scan(p, 20000, cfg)
    with pytest.raises(UnboundLocalError):
        cli.main(base + ["--window", "20000"])
    outs = cli.main(base + ["--window", "500000", "--window", "1000000", "--snp-window", "100"])
    assert [os.path.basename(o) for o in outs] == ["run_500kb.csv", "run_1000kb.csv", "run_100snps.csv"]
    for path, ref in ((outs[0], O.combined_scan(p, 500000, cfg)), (outs[1], O.combined_scan(p, 1000000, cfg))):
        rows = _read(path)
        assert len(rows) == len(ref)
        for r, (label, o) in zip(rows, ref.items()):
            chrom, span = label.split(" ")
            assert (r["chromosome"], f"{r['window_start']}-{r['window_end']}") == (chrom, span)
            assert int(r["snp_count"]) == o["snp_count"]
            for f, g in (("T2D", "T2D"), ("T1D_p1", "T1D_pop1"), ("T1D_p2", "T1D_pop2")):
                if o[g] is None:
                    assert r[f] == ""
                else:
                    assert close(float(r[f]), o[g])
            s, e = int(r["window_start"]), int(r["window_end"])
            c = p.chrom_names.index(chrom)
            lo, hi = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
            idx = np.arange(lo, hi)[(p.pos[lo:hi] >= s) & (p.pos[lo:hi] <= e)]
            f = O.window_fst(p, idx, cfg)
            assert (r["FST"] == "") if f is None else abs(float(r["FST"]) - f) <= 1e-9 * max(1.0, abs(f))
    ref = O.scan_perChr_bySNPs(p, 100, cfg)
    rows = _read(outs[2])
    assert [f"{r['chromosome']} {r['window_start']}-{r['window_end']}" for r in rows] == list(ref)
    for r, o in zip(rows, ref.values()):
        assert close(float(r["T2D"]), o["T2D"]) and close(float(r["T2D_diff"]), o["T2D_diff"], scale=abs(o["T2D"]))
