"""Command line: VCF + popmap in, per-window statistics CSV out.

The reference's entry point is the notebook-style script at the bottom of
scripts/src/twoDSFS_class.py (1788-2040): load the SNP dict, run ``combined_scan`` at 20 kb and
500 kb and ``scan_perChr_bySNPs`` at 500 / 300 SNPs, and write each result with
``save_csv_stats`` (1884-1907; chromosome accessions renamed through chromosomes.txt, 1788-1797).
This CLI runs the same drivers on the GPU path, from the native VCF parser straight to the packed
arrays (no dict), every window size from one resident upload and one k_prep pass (multi_scan):

    python -m sfs2d VCF POPMAP --window 20000 --window 500000 --snp-window 500 \\
        --chromosomes chromosomes.txt --out-prefix ECBstats [--fst | --pixy-fst fst_20kb.csv]

Outputs ``<prefix>_20kb.csv``, ``<prefix>_500kb.csv``, ``<prefix>_500snps.csv`` with the reference's
columns; ``--fst`` appends an ``FST`` column with this framework's Hudson estimator,
``--pixy-fst FILE`` instead joins pixy's ``avg_wc_fst`` by (chromosome, window_start,
window_end) the way ECBstats_plots.R:16-41 does (pixy chromosome ``NC_087088_1`` -> ``NC_087088.1``)
-- the FST column of the published data/ECBstats_*.csv.
"""
from __future__ import annotations

import argparse
import csv
import os
import re
import sys
import time


def _fmt_kb(ws: int) -> str:
    return f"{ws // 1000}kb" if ws % 1000 == 0 else f"{ws}bp"


def read_pixy_fst(path):
    """pixy windowed Fst CSV -> {(accession, start, end): avg_wc_fst} (ECBstats_plots.R:16-28)."""
    out = {}
    with open(path, newline="", encoding="utf-8-sig") as fh:
        for row in csv.DictReader(fh):
            chrom = re.sub(r"^(.*?_.*?)_(.*)$", r"\1.\2", row["chromosome"])
            v = row["avg_wc_fst"]
            out[(chrom, str(row["window_pos_1"]), str(row["window_pos_2"]))] = None if v in ("", "NA") else float(v)
    return out


def write_csv(path, stats, chr_ids, fst=None, pixy=None):
    """save_csv_stats (twoDSFS_class.py:1884-1907) + optional FST column."""
    import twoDSFS_class as T
    cols = list(T.col_names) + (["FST"] if (fst is not None or pixy is not None) else [])
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=cols)
        w.writeheader()
        for label, r in stats.items():
            chrom = label.split(" ")[0]
            s, e = label.split(" ")[1].split("-")
            row = {"chromosome": chr_ids.get(chrom, chrom), "window_start": s, "window_end": e,
                   "snp_count": r["snp_count"], "T2D": r["T2D"], "T1D_p1": r["T1D_pop1"], "T1D_p2": r["T1D_pop2"],
                   "new_term_p1": r["new_term_pop1"], "new_term_p2": r["new_term_pop2"],
                   "T2D_diff": r.get("T2D_diff")}
            if fst is not None:
                row["FST"] = fst.get(label)
            elif pixy is not None:
                row["FST"] = pixy.get((chrom, s, e))
            w.writerow(row)


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m sfs2d", description=__doc__.split("\n\n")[0])
    ap.add_argument("vcf")
    ap.add_argument("popmap")
    ap.add_argument("--pop1", default="uv")
    ap.add_argument("--pop2", default="bv")
    ap.add_argument("--pop1-size", type=int, default=18, help="diploid individuals of pop1 (twoDSFS_class.py:22)")
    ap.add_argument("--pop2-size", type=int, default=14)
    ap.add_argument("--window", type=int, action="append", default=[], help="fixed-bp window (combined_scan)")
    ap.add_argument("--snp-window", type=int, action="append", default=[], help="SNPs per window (scan_perChr_bySNPs)")
    ap.add_argument("--variant-type", default=None)
    ap.add_argument("--no-fold", action="store_true")
    ap.add_argument("--chromosomes", default=None, help="accession<TAB>number map (chromosomes.txt)")
    ap.add_argument("--fst", action="store_true", help="append Hudson's Fst (this framework's estimator)")
    ap.add_argument("--pixy-fst", default=None, help="join pixy avg_wc_fst as the FST column")
    ap.add_argument("--out-prefix", default="stats")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--threads", type=int, default=0, help="VCF parser threads (0 = all)")
    a = ap.parse_args(argv)
    if not a.window and not a.snp_window:
        a.window = [20000]

    import twoDSFS_class as T
    from sfs2d.vcf import make_packed_vcf

    t0 = time.perf_counter()
    packed = make_packed_vcf(a.vcf, a.popmap, a.pop1, a.pop2, nthreads=a.threads)
    t1 = time.perf_counter()
    print(f"ingest: {packed.n} SNPs, {packed.nchrom} chromosomes in {t1 - t0:.3f} s", file=sys.stderr)
    chr_ids = T.load_chr_ids(a.chromosomes) if a.chromosomes else {}
    pixy = read_pixy_fst(a.pixy_fst) if a.pixy_fst else None
    obj = T.LikelihoodInference_jointSFS(a.vcf, a.popmap, pop1=a.pop1, pop2=a.pop2, pop1_size=a.pop1_size,
                                         pop2_size=a.pop2_size, variant_type=a.variant_type, fold=not a.no_fold,
                                         device=a.device)
    outs = []
    t = time.perf_counter()
    # every window size from one k_prep pass over the resident stream (sfs2d_plan_attach)
    res = obj.multi_scan(packed, a.window, a.snp_window, fst=a.fst)
    print(f"multi_scan ({len(a.window)} bp + {len(a.snp_window)} SNP-count window sizes): "
          f"{time.perf_counter() - t:.2f} s", file=sys.stderr)
    for ws in a.window:
        path = f"{a.out_prefix}_{_fmt_kb(ws)}.csv"
        write_csv(path, res[ws], chr_ids, res["fst"][ws] if a.fst else None, pixy)
        outs.append(path)
        print(f"combined_scan {ws} bp: {len(res[ws])} windows -> {path}", file=sys.stderr)
    for S in a.snp_window:
        stats = res[f"{S}snps"]
        fst = obj.window_fst(packed, snp_window_size=S) if a.fst else None
        path = f"{a.out_prefix}_{S}snps.csv"
        write_csv(path, stats, chr_ids, fst, pixy)
        outs.append(path)
        print(f"scan_perChr_bySNPs {S} SNPs: {len(stats)} windows -> {path}", file=sys.stderr)
    return outs


if __name__ == "__main__":
    main()
