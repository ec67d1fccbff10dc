"""Sims batch driver (sims_scan.process_windows_batch / likelihood_scan): many replicates scanned in
one launch against one generation background must equal the reference's per-replicate
process_window (sims_scan.py:451-590; golden sims_n10 / sims_n100 from the reference itself) and the
oracle's restatement on synthetic replicates; likelihood_scan end to end over a directory of VCFs."""
import csv
import gzip
import os

import numpy as np
import pytest

import golden_util as gu

pytestmark = pytest.mark.gpu


def _bg(S, bgd, n):
    return (S.calculate_2d_sfs(bgd, "p1", "p2", n, n, start_position=0, end_position=500000, variant_type=None),
            S.calculate_1d_sfs(bgd, "p1", n, start_position=0, end_position=500000, variant_type=None),
            S.calculate_1d_sfs(bgd, "p2", n, start_position=0, end_position=500000, variant_type=None))


@pytest.mark.parametrize("tag", ["sims_n10", "sims_n100"])
def test_batch_golden(golden, tag):
    import sims_scan as S
    from sfs2d.synth import synth_genome
    rep = golden.packed(tag)
    n = golden.cfg(tag)["n1p"]
    bg = _bg(S, golden.packed(f"{tag}_bgdata"), n)
    ref = gu.decode_results(golden.calls(tag)[0]["out"]["results"])
    extra = synth_genome(2, [4000, 2500], n, n, seed=3, chrom_prefix="1.")
    outs = S.process_windows_batch([rep, extra, rep], *bg, 500000, "p1", "p2", n, n)
    assert not gu.compare_results(outs[0], ref) and not gu.compare_results(outs[2], ref)
    # (n = 100 takes the large-grid path, whose exact re-evaluations sum in the order in which lanes
    # win the histogram take-and-clear: equal within the tolerance, not bit for bit)
    assert not gu.compare_results(outs[1], S.process_window(extra, *bg, 500000, "p1", "p2", n, n, None, None, None))


def test_batch_vs_oracle_and_errors():
    import sims_scan as S
    from oracle import sfs_oracle as O
    from sfs2d.synth import synth_genome
    n = 5
    bgd = synth_genome(1, 30000, n, n, seed=11, chrom_prefix="1")
    bg = _bg(S, bgd, n)
    o2, o1, o1b = O.sims_backgrounds(bgd, n, n)
    reps = [synth_genome(1 + (i % 2), [20000 + 977 * i] * (1 + (i % 2)), n, n, seed=100 + i, chrom_prefix="1")
            for i in range(6)]
    outs = S.process_windows_batch(reps, *bg, 500000, "p1", "p2", n, n)
    for r, out in zip(reps, outs):
        ref = O.sims_process_window(r, o2, o1, o1b, 500000, n, n)
        assert not gu.compare_results(out, ref)
    # an empty window: the replicate raises as the reference's process_window would
    empty = synth_genome(1, 5, n, n, seed=1, chrom_prefix="1")
    empty.counts[:] = 0
    with pytest.raises(ZeroDivisionError):
        S.process_windows_batch(reps[:2] + [empty], *bg, 500000, "p1", "p2", n, n)


def _write_vcf(path, packed, samples_p1, samples_p2):
    """A replicate as a VCF whose genotypes reproduce the packed allele counts (p1 / p2 samples)."""
    lines = ["##fileformat=VCFv4.2",
             "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples_p1 + samples_p2)]
    ch = packed.chrom_of()
    for i in range(packed.n):
        gts = []
        for (r, a), ns in (((packed.ref1[i], packed.alt1[i]), len(samples_p1)),
                           ((packed.ref2[i], packed.alt2[i]), len(samples_p2))):
            alle = ["1"] * int(a) + ["0"] * int(r)
            alle += ["."] * (2 * ns - len(alle))
            gts += [f"{alle[2 * k]}/{alle[2 * k + 1]}" for k in range(ns)]
        lines.append(f"{packed.chrom_names[ch[i]]}\t{int(packed.pos[i])}\t.\tA\tG\t.\tPASS\tPR\tGT\t" + "\t".join(gts))
    with gzip.open(path, "wt") as fh:
        fh.write("\n".join(lines) + "\n")


def test_likelihood_scan_end_to_end(tmp_path):
    import sims_scan as S
    from oracle import sfs_oracle as O
    from sfs2d.synth import synth_genome
    n = 5
    s1, s2 = [f"a{i}" for i in range(n)], [f"b{i}" for i in range(n)]
    popmap = tmp_path / "popmap.txt"
    popmap.write_text("".join(f"{s}\tp1\n" for s in s1) + "".join(f"{s}\tp2\n" for s in s2))
    (tmp_path / "concatenated_vcfs").mkdir()
    bgd = synth_genome(1, 40000, n, n, seed=5, chrom_prefix="1")
    _write_vcf(tmp_path / "concatenated_vcfs" / "gen.2000.concatenated.vcf.gz", bgd, s1, s2)
    reps = {}
    for it in (3, 7, 12):
        d = tmp_path / f"iter{it}"
        d.mkdir()
        reps[it] = synth_genome(1, 30000, n, n, seed=it, chrom_prefix="1")
        _write_vcf(d / f"rep.2000.{it}.vcf.gz", reps[it], s1, s2)
    out = tmp_path / "res.csv"
    S.likelihood_scan(str(tmp_path), str(out), str(popmap), "p1", "p2", n, n)
    rows = list(csv.DictReader(open(out)))
    o2, o1, o1b = O.sims_backgrounds(bgd, n, n)
    got = {}
    for r in rows:
        got.setdefault(int(r["iteration"]), []).append(r)
    assert sorted(got) == [3, 7, 12]
    for it, rs in got.items():
        ref = O.sims_process_window(reps[it], o2, o1, o1b, 500000, n, n)
        assert [r["window_coords"] for r in rs] == list(ref)
        for r, (k, o) in zip(rs, ref.items()):
            assert r["generation"] == "2000" and int(r["snp_count"]) == o["snp_count"]
            assert r["region"] == ("background" if int(k.split(" ")[1].split("-")[1]) <= 1000000 else "foreground")
            for f in ("T2D", "T1D_p1", "T1D_p2"):
                assert gu.close(float(r[f]), o[f])
            assert gu.close(float(r["T2D_diff"]), o["T2D_diff"], scale=abs(o["T2D"]))


def test_likelihood_scan_dict_variant(tmp_path):
    """sims_scan.py:646-690 (the definition the reference module keeps): the dict keyed by
    (generation, iteration, window) whose 'likelihood' is process_window's record, equal to the CSV
    variant's rows and to the oracle."""
    import sims_scan as S
    from oracle import sfs_oracle as O
    from sfs2d.synth import synth_genome
    n = 5
    s1, s2 = [f"a{i}" for i in range(n)], [f"b{i}" for i in range(n)]
    popmap = tmp_path / "popmap.txt"
    popmap.write_text("".join(f"{s}\tp1\n" for s in s1) + "".join(f"{s}\tp2\n" for s in s2))
    (tmp_path / "concatenated_vcfs").mkdir()
    bgd = synth_genome(1, 30000, n, n, seed=6, chrom_prefix="1")
    _write_vcf(tmp_path / "concatenated_vcfs" / "gen.500.concatenated.vcf.gz", bgd, s1, s2)
    reps = {}
    for it in (1, 4):
        d = tmp_path / f"iter{it}"
        d.mkdir()
        reps[it] = synth_genome(1, 20000, n, n, seed=40 + it, chrom_prefix="1")
        _write_vcf(d / f"rep.500.{it}.vcf.gz", reps[it], s1, s2)
    got = S.likelihood_scan(str(tmp_path), popinfo_filename=str(popmap))
    o2, o1, o1b = O.sims_backgrounds(bgd, n, n)
    want_keys = []
    for it in sorted(reps):
        ref = O.sims_process_window(reps[it], o2, o1, o1b, 500000, n, n)
        for k, o in ref.items():
            want_keys.append(("500", it, k))
            v = got[("500", it, k)]
            assert v["generation"] == "500" and v["iteration"] == it and v["window_coords"] == k
            assert v["region"] == ("background" if int(k.split(" ")[1].split("-")[1]) <= 1000000 else "foreground")
            assert not gu.compare_results({k: v["likelihood"]}, {k: o})
    assert sorted(got) == sorted(want_keys)
    with pytest.raises(FileNotFoundError):
        S.likelihood_scan(str(tmp_path), popinfo_filename=str(tmp_path / "absent.txt"))
