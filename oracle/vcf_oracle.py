"""TEST INFRASTRUCTURE ONLY (the oracle): VCF(.gz) + popmap -> SNP dict in plain Python.

Checker for the native parser (2dsfs-scan_amd/csrc/vcf_ingest.cpp, include/sfs2d_ingest.h);
only tests/ may import it.  Pinned by tests/golden/vcf_expected_*.npz, produced by the
reference's own make_data_dict_vcf (tests/golden/gen_golden_vcf.py).

Restates ``make_data_dict_vcf`` (twoDSFS_class.py:36-138; sims_scan.py:18-120), including its
quirks:

* popmap: tab-separated ``sample<TAB>pop``; lines with fewer than 2 columns are ignored (57-64);
* ``poplist`` holds the popmap label of every header sample FOUND in the popmap, in header order,
  and is then zipped POSITIONALLY against all sample columns (81-85, 118): unmapped samples
  shift the labels;
* FILTER must be ``PASS`` or ``.`` (101-102); REF and ALT must each be one of A/C/G/T after
  upper-casing (104-109); annotation is the 2nd '|' field of INFO, else ``'No annotation'``;
* per sample, alleles are counted as ``gt[::2].count('0')`` / ``.count('1')`` (128-129);
* keys are ``CHROM-POS`` strings; a repeated key keeps the last record (dict assignment).
"""
from __future__ import annotations

import gzip


def read_popmap(popinfo_filename):
    popmap = {}
    with open(popinfo_filename, "r") as fh:
        for line in fh:
            columns = line.strip().split("\t")
            if len(columns) >= 2:
                popmap[columns[0]] = columns[1]
    return popmap


def make_data_dict_vcf(vcf_filename, popinfo_filename):
    popmap = read_popmap(popinfo_filename)
    data_dict = {}
    poplist = []
    opener = gzip.open if str(vcf_filename).endswith((".gz", ".bgz")) else open
    with opener(vcf_filename, "rt") as vcf_file:
        for line in vcf_file:
            if line.startswith("##"):
                continue
            if line.startswith("#"):
                for sample in line.split()[9:]:
                    if sample in popmap:
                        poplist.append(popmap[sample])
                continue
            cols = line.split("\t")
            snp_id = "-".join(cols[:2])
            parts = cols[7].split("|")
            annotation = parts[1] if len(parts) >= 2 else "No annotation"
            if cols[6] != "PASS" and cols[6] != ".":
                continue
            ref = cols[3].upper()
            alt = cols[4].upper()
            if ref not in ("A", "C", "G", "T") or alt not in ("A", "C", "G", "T"):
                continue
            gtindex = cols[8].split(":").index("GT")
            calls = {}
            for pop, sample in zip(poplist, cols[9:]):
                if pop is None:
                    continue
                gt = sample.split(":")[gtindex]
                r, a = calls.get(pop, (0, 0))
                calls[pop] = (r + gt[::2].count("0"), a + gt[::2].count("1"))
            data_dict[snp_id] = {"segregating": (ref, alt), "context": "-" + ref + "-",
                                 "calls": calls, "annotation": annotation}
    return data_dict
