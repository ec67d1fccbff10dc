#!/usr/bin/env python3
"""Golden vectors for the VCF + popmap ingest (build container only; reads /root/reference).

Input: a test VCF assembled from the first records of the reference's own data file
``vcf_pruned/ECB_LDprunedv2.vcf.gz`` (header + 2500 records, data only) followed by hand-made
records that exercise every rule of ``make_data_dict_vcf`` (twoDSFS_class.py:36-138): FILTER
values (101-102), multi-allelic / symbolic / lower-case alleles (104-109), INFO annotations
(92-97), GT not first in FORMAT (115), phased / haploid / missing genotypes (120-130), duplicate
CHROM-POS keys (the last record that passes the filters wins; a failing duplicate changes
nothing), a position with a leading zero (a distinct dict key at the same integer position).
The reference's ``popmap.txt`` (CRLF line ends; IDs that do not match the v2 header: quirk Q12)
and a second popmap with three populations are the population maps.

Expected outputs come from the REFERENCE's own ``make_data_dict_vcf`` run unmodified (loaded as in
gen_golden.py); only data is written: the test VCF in two encodings (BGZF, one-member gzip;
the tests decompress it for the plain-text case), the popmaps, and ``vcf_expected_<popmap>.npz`` with the dict flattened to arrays.
A digest of the full ECB_LDprunedv2.vcf.gz result is stored too (checked only where the
reference data exists).

Run:  python tests/golden/gen_golden_vcf.py
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import struct
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen_golden import REF, load_reference_module  # noqa: E402

N_REAL = 2500


def bgzf_bytes(data: bytes, block: int = 65280) -> bytes:
    """BGZF (SAM spec 4.1): gzip members of <= 64 KiB with the 'BC' extra field, then the EOF block."""
    out = bytearray()
    for i in range(0, len(data) + 1, block):
        chunk = data[i:i + block]
        if not chunk and i:
            break
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        cdata = c.compress(chunk) + c.flush()
        bsize = 18 + len(cdata) + 8
        out += b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<H", 6) + b"BC" + \
            struct.pack("<HH", 2, bsize - 1) + cdata + struct.pack("<II", zlib.crc32(chunk), len(chunk))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


def crafted(samples):
    """Hand-made records (tab-separated), each a rule of make_data_dict_vcf."""
    ns = len(samples)

    def gts(pattern):
        return "\t".join(pattern[i % len(pattern)] for i in range(ns))
    chrom_a, chrom_b = "NC_087088.1", "NC_087089.1"
    rec = []
    rec.append(f"{chrom_a}\t9000001\t.\tA\tG\t.\tLowQual\tPR\tGT\t{gts(['0/1', '1/1'])}")          # FILTER fails
    rec.append(f"{chrom_a}\t9000002\t.\tA\tG,T\t.\tPASS\tPR\tGT\t{gts(['0/1', '0/2'])}")           # multi-allelic
    rec.append(f"{chrom_a}\t9000003\t.\tA\t<DEL>\t.\t.\tPR\tGT\t{gts(['0/1'])}")                   # symbolic
    rec.append(f"{chrom_a}\t9000004\t.\tAT\tA\t.\t.\tPR\tGT\t{gts(['0/1'])}")                      # indel
    rec.append(f"{chrom_a}\t9000005\t.\ta\tc\t.\tPASS\tPR\tGT\t{gts(['0/1', '0/0', '1/1', './.'])}")  # lower case
    rec.append(f"{chrom_a}\t9000006\t.\tC\tT\t.\t.\tANN=T|missense_variant|MODERATE\tGT\t{gts(['0|1', '1|0', '0|0'])}")
    rec.append(f"{chrom_a}\t9000007\t.\tG\tA\t.\t.\tANN=A|synonymous_variant\tGT\t{gts(['0/0', '0/1'])}")
    rec.append(f"{chrom_a}\t9000008\t.\tG\tA\t.\t.\tX=1|\tGT\t{gts(['0/1'])}")                     # empty annotation
    rec.append(f"{chrom_a}\t9000009\t.\tT\tC\t.\t.\tPR\tDP:GT\t{gts(['7:0/1', '3:1/1', '0:./.'])}")  # GT second
    rec.append(f"{chrom_a}\t9000010\t.\tT\tC\t.\t.\tPR\tGT:DP\t{gts(['1:4', '0:2', '.:0'])}")       # haploid
    rec.append(f"{chrom_a}\t9000011\t.\tT\tG\t.\t.\tPR\tGT\t{gts(['1/1', '0/1'])}")
    rec.append(f"{chrom_a}\t9000011\t.\tT\tG\t.\t.\tPR\tGT\t{gts(['0/0', '0/1', '1/1'])}")          # duplicate: wins
    rec.append(f"{chrom_a}\t9000012\t.\tT\tG\t.\t.\tPR\tGT\t{gts(['0/1'])}")
    rec.append(f"{chrom_a}\t9000012\t.\tT\tG\t.\tq10\tPR\tGT\t{gts(['1/1'])}")                      # failing duplicate
    rec.append(f"{chrom_a}\t09000013\t.\tC\tG\t.\t.\tPR\tGT\t{gts(['0/1', '1/1'])}")               # leading zero
    rec.append(f"{chrom_a}\t9000013\t.\tC\tG\t.\t.\tPR\tGT\t{gts(['0/0', '0/1'])}")                # same int position
    rec.append(f"{chrom_b}\t15\t.\tG\tC\t.\tPASS\tPR\tGT\t{gts(['0/1', '1/1', '0/0'])}")           # a later chromosome
    rec.append(f"{chrom_a}\t5\t.\tG\tC\t.\tPASS\tPR\tGT\t{gts(['0/1'])}")                          # out of order
    rec.append(f"{chrom_b}\t154450\t.\tG\tT\t.\t.\tPR\tGT\t{gts(['1/1', '0/1', '0/0', '1|1'])}")
    return rec


def flatten(d):
    """dict -> arrays (the dict's insertion order): keys, segregating, context, annotation, calls per pop."""
    keys = list(d.keys())
    pops = []
    for v in d.values():
        for p in v["calls"]:
            if p not in pops:
                pops.append(p)
    calls = np.full((len(keys), len(pops), 2), -1, dtype=np.int64)
    for i, k in enumerate(keys):
        for p, (r, a) in d[k]["calls"].items():
            calls[i, pops.index(p)] = (r, a)
    return {
        "keys": np.array(keys, dtype=str),
        "seg_ref": np.array([d[k]["segregating"][0] for k in keys], dtype=str),
        "seg_alt": np.array([d[k]["segregating"][1] for k in keys], dtype=str),
        "context": np.array([d[k]["context"] for k in keys], dtype=str),
        "annotation": np.array([d[k]["annotation"] for k in keys], dtype=str),
        "pops": np.array(pops, dtype=str),
        "calls": calls,
        # the order in which each record's calls dict lists its populations
        "call_order": np.array(["\t".join(d[k]["calls"].keys()) for k in keys], dtype=str),
    }


def digest(d):
    h = hashlib.sha256()
    for k, v in d.items():
        h.update(repr((k, v["segregating"], v["context"], v["annotation"], list(v["calls"].items()))).encode())
    return h.hexdigest()


def main():
    mod = load_reference_module(f"{REF}/scripts/src/twoDSFS_class.py", "ref_twoDSFS_class")
    obj = mod.LikelihoodInference_jointSFS(None, None)
    src = f"{REF}/vcf_pruned/ECB_LDprunedv2.vcf.gz"
    with gzip.open(src, "rt") as fh:
        lines = fh.read().split("\n")
    head = [ln for ln in lines if ln.startswith("#")]
    body = [ln for ln in lines if ln and not ln.startswith("#")]
    samples = head[-1].split()[9:]
    text = "\n".join(head + body[:N_REAL] + crafted(samples)) + "\n"
    raw = text.encode()
    with open(os.path.join(HERE, "vcf_test.vcf.gz"), "wb") as fh:
        fh.write(bgzf_bytes(raw))
    with open(os.path.join(HERE, "vcf_test_plain.vcf.gz"), "wb") as fh:
        fh.write(gzip.compress(raw, 6, mtime=0))
    with open(f"{REF}/popmap.txt", "rb") as fh:
        pm = fh.read()
    with open(os.path.join(HERE, "popmap_ref.txt"), "wb") as fh:
        fh.write(pm)
    # a second map: v2 header IDs, three populations, one sample unmapped, one line malformed
    pm3 = []
    for i, s in enumerate(samples):
        if i == 5:
            continue
        pm3.append(f"{s}\t{['uv', 'bv', 'zz'][i % 3]}")
    pm3.insert(3, "lonely_line_without_tab")
    with open(os.path.join(HERE, "popmap_3pop.txt"), "w") as fh:
        fh.write("\n".join(pm3) + "\n")
    manifest = {}
    for name in ("popmap_ref", "popmap_3pop"):
        for vcf in ("vcf_test.vcf.gz", "vcf_test_plain.vcf.gz"):
            d = obj.make_data_dict_vcf(os.path.join(HERE, vcf), os.path.join(HERE, f"{name}.txt"))
            if vcf == "vcf_test.vcf.gz":
                np.savez_compressed(os.path.join(HERE, f"vcf_expected_{name}.npz"), **flatten(d))
                manifest[name] = {"records": len(d), "digest": digest(d)}
            else:
                assert digest(d) == manifest[name]["digest"], "gzip encodings disagree"
        print(name, len(d), "records")
    full = obj.make_data_dict_vcf(src, f"{REF}/popmap.txt")
    manifest["full_ECB_LDprunedv2"] = {"records": len(full), "digest": digest(full),
                                       "note": "reference vcf_pruned/ECB_LDprunedv2.vcf.gz + popmap.txt"}
    print("full", len(full))
    with open(os.path.join(HERE, "vcf_manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)


if __name__ == "__main__":
    main()
