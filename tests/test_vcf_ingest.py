"""Native VCF + popmap ingest (include/sfs2d_ingest.h) against the reference's make_data_dict_vcf.

Pinned by tests/golden/vcf_expected_*.npz, written by the reference's own function
(tests/golden/gen_golden_vcf.py; twoDSFS_class.py:36-138).  Larger and adversarial inputs are
checked against oracle/vcf_oracle.py (the Python restatement, itself pinned by the same goldens).
CPU only: the parser is host code.
"""
import gzip
import json
import os
import re
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
sys.path.insert(0, REPO)
GOLD = os.path.join(HERE, "golden")

from oracle import vcf_oracle  # noqa: E402
from sfs2d import vcf as V  # noqa: E402
from sfs2d.pack import pack_snp_dict  # noqa: E402

pytestmark = pytest.mark.skipif(not os.path.exists(V.INGEST_PATH), reason="libsfs2d_ingest.so not built")


def flatten(d):
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
    return {"keys": keys, "seg_ref": [d[k]["segregating"][0] for k in keys],
            "seg_alt": [d[k]["segregating"][1] for k in keys], "context": [d[k]["context"] for k in keys],
            "annotation": [d[k]["annotation"] for k in keys], "pops": pops, "calls": calls,
            "call_order": ["\t".join(d[k]["calls"].keys()) for k in keys]}


def same_dict(a, b):
    assert list(a.keys()) == list(b.keys())
    for k in a:
        assert a[k] == b[k], k
        assert list(a[k].keys()) == list(b[k].keys())
        assert list(a[k]["calls"].keys()) == list(b[k]["calls"].keys())


def test_exports_match_header():
    import ctypes
    hdr = open(os.path.join(REPO, "include", "sfs2d_ingest.h")).read()
    declared = sorted(set(re.findall(r"\b(sfs2d_vcf_\w+)\s*\(", hdr)))
    assert declared == sorted(V.EXPORTS)
    lib = ctypes.CDLL(V.INGEST_PATH)
    for name in declared:
        assert hasattr(lib, name), name


@pytest.mark.parametrize("popmap", ["popmap_ref", "popmap_3pop"])
@pytest.mark.parametrize("enc", ["bgzf", "gzip", "text", "crlf"])
def test_golden(popmap, enc, tmp_path):
    src = os.path.join(GOLD, "vcf_test.vcf.gz")
    if enc == "gzip":
        path = os.path.join(GOLD, "vcf_test_plain.vcf.gz")
    elif enc == "bgzf":
        path = src
    else:
        raw = gzip.open(src, "rb").read()
        if enc == "crlf":
            raw = raw.replace(b"\n", b"\r\n")
        path = str(tmp_path / "t.vcf")
        open(path, "wb").write(raw)
    exp = np.load(os.path.join(GOLD, f"vcf_expected_{popmap}.npz"))
    for nt in (1, 4):
        got = flatten(V.read_vcf(path, os.path.join(GOLD, f"{popmap}.txt"), nthreads=nt).to_data_dict())
        for f in ("keys", "seg_ref", "seg_alt", "context", "annotation", "pops", "call_order"):
            assert list(got[f]) == exp[f].tolist(), f
        assert np.array_equal(got["calls"], exp["calls"])
    man = json.load(open(os.path.join(GOLD, "vcf_manifest.json")))
    assert len(got["keys"]) == man[popmap]["records"]


def test_packed_matches_dict_packing():
    path, pm = os.path.join(GOLD, "vcf_test.vcf.gz"), os.path.join(GOLD, "popmap_3pop.txt")
    t = V.read_vcf(path, pm)
    for p1, p2 in (("uv", "bv"), ("zz", "uv"), ("uv", "nope")):
        a = t.to_packed(p1, p2)
        b = pack_snp_dict(vcf_oracle.make_data_dict_vcf(path, pm), p1, p2)
        assert np.array_equal(a.counts, b.counts) and np.array_equal(a.pos, b.pos)
        assert np.array_equal(a.chrom_off, b.chrom_off) and a.chrom_names == b.chrom_names
        assert [a.ann_names[i] for i in a.ann_id] == [b.ann_names[i] for i in b.ann_id]


def synth_vcf(n, samples, seed, dup_every=97, late_header=False, bad=None):
    """A larger VCF (several parse chunks) with duplicates, filters, formats, CRLF/CR line ends."""
    rng = np.random.default_rng(seed)
    head = ["##fileformat=VCFv4.2", "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples)]
    gts = np.array(["0/0", "0/1", "1/1", "./.", "0|1", "1", "1/0", "0/2"])
    lines = []
    for i in range(n):
        chrom = f"chr{int(rng.integers(1, 4))}"
        pos = int(rng.integers(1, 50000)) if i % dup_every else int(lines[-1].split("\t")[1]) if lines else 7
        if i % dup_every == 0 and lines:
            chrom = lines[-1].split("\t")[0]
        filt = ["PASS", ".", "LowQual"][int(rng.integers(0, 3)) if i % 5 == 0 else 0]
        ref, alt = ("A", "C") if i % 7 else (("g", "t") if i % 2 else ("A", "C,T"))
        info = "ANN=x|" + ["syn", "mis", "intron"][i % 3] if i % 4 else "DP=3"
        fmt, g = ("GT", gts[rng.integers(0, len(gts), len(samples))]) if i % 6 else \
            ("DP:GT", [f"{int(d)}:{x}" for d, x in zip(rng.integers(0, 9, len(samples)),
                                                       gts[rng.integers(0, len(gts), len(samples))])])
        lines.append(f"{chrom}\t{pos}\t.\t{ref}\t{alt}\t.\t{filt}\t{info}\t{fmt}\t" + "\t".join(g))
        if late_header and i == n // 2:
            lines.append("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples[::-1]))
    if bad is not None:
        lines.insert(bad[0], bad[1])
    text = "\n".join(head + lines) + "\n"
    return text.replace("\n", "\r\n", 50).encode()   # a few CRLF line ends at the top


SAMPLES = [f"s{i}" for i in range(24)]


def write_popmap(path, mapping):
    open(path, "w").write("".join(f"{s}\t{p}\n" for s, p in mapping))


@pytest.mark.parametrize("late,merge_chunk", [(False, None), (True, None), (False, "97")])
def test_threads_and_oracle(tmp_path, monkeypatch, late, merge_chunk):
    """Thread-count independence; merge_chunk: the dict merge sharded over many threads (97-record
    shards instead of 64k) -- duplicate keys across shards and parse chunks keep dict semantics."""
    if merge_chunk:
        monkeypatch.setenv("SFS2D_VCF_MERGE_CHUNK", merge_chunk)
    raw = synth_vcf(40000, SAMPLES, seed=5, late_header=late)
    path = str(tmp_path / "s.vcf.gz")
    open(path, "wb").write(gzip.compress(raw, 1))
    pm = str(tmp_path / "pm.txt")
    write_popmap(pm, [(s, ["uv", "bv", "x"][i % 3]) for i, s in enumerate(SAMPLES) if i != 4])
    ref = vcf_oracle.make_data_dict_vcf(path, pm)
    for nt in (1, 2, 7, 16):
        same_dict(V.read_vcf(path, pm, nthreads=nt).to_data_dict(), ref)


def test_merge_skewed_shards(tmp_path, monkeypatch):
    """Every key hashed into one shard of a many-shard merge: that shard's table is sized from its own
    record count (a table sized from total / shards filled up and its probe never ended)."""
    monkeypatch.setenv("SFS2D_VCF_MERGE_CHUNK", "61")
    monkeypatch.setenv("SFS2D_VCF_MERGE_SKEW", "1")
    raw = synth_vcf(8000, SAMPLES, seed=11)
    path = str(tmp_path / "k.vcf")
    open(path, "wb").write(raw)
    pm = str(tmp_path / "pm.txt")
    write_popmap(pm, [(s, ["uv", "bv"][i % 2]) for i, s in enumerate(SAMPLES)])
    ref = vcf_oracle.make_data_dict_vcf(path, pm)
    for nt in (4, 16):
        same_dict(V.read_vcf(path, pm, nthreads=nt).to_data_dict(), ref)


def sorted_vcf(n, samples, seed, twist=None):
    """A VCF in (chromosome, position) order -- the parser's no-merge fast path -- or, with twist, one
    that breaks exactly one of that path's conditions (so the hash merge must take over)."""
    rng = np.random.default_rng(seed)
    head = ["##fileformat=VCFv4.2", "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples)]
    gts = np.array(["0/0", "0/1", "1/1", "./.", "1/0"])
    lines, per = [], n // 3
    for c in range(3):
        pos = np.cumsum(rng.integers(1, 40, per))
        for q in pos.tolist():
            g = gts[rng.integers(0, len(gts), len(samples))]
            lines.append([f"chr{c + 1}", str(q), ".", "A", "G", ".", "PASS", "ANN=x|syn", "GT"] + list(g))
    m = len(lines) // 2
    if twist == "dup":              # a repeated key (dict semantics: first slot, last values)
        lines[m][1] = lines[m - 1][1]
    elif twist == "zero":           # "0<pos>": another key, the same integer position
        lines[m][1] = "0" + lines[m - 1][1]
    elif twist == "back":           # chr1 again after chr2
        lines.insert(2 * per - 5, ["chr1", str(10 ** 9)] + lines[0][2:])
    elif twist == "text":           # a position that is not a plain decimal
        lines[m][1] = lines[m][1] + "x"
    return ("\n".join(head + ["\t".join(x) for x in lines]) + "\n").encode()


@pytest.mark.parametrize("twist", [None, "dup", "zero", "back", "text"])
def test_sorted_fast_path(tmp_path, monkeypatch, twist):
    """Sorted files skip the dict merge (no key can repeat); files breaking any of its conditions
    take the hash merge.  Both agree with the oracle and with the forced hash merge."""
    raw = sorted_vcf(60000, SAMPLES, seed=21, twist=twist)   # > 1 MB: several parse chunks
    path = str(tmp_path / "o.vcf")
    open(path, "wb").write(raw)
    pm = str(tmp_path / "pm.txt")
    write_popmap(pm, [(s, ["uv", "bv"][i % 2]) for i, s in enumerate(SAMPLES)])
    ref = vcf_oracle.make_data_dict_vcf(path, pm)
    for nt in (1, 5):
        same_dict(V.read_vcf(path, pm, nthreads=nt).to_data_dict(), ref)
    monkeypatch.setenv("SFS2D_VCF_HASH_MERGE", "1")
    same_dict(V.read_vcf(path, pm, nthreads=5).to_data_dict(), ref)
    if twist != "text":
        a = V.read_vcf(path, pm, nthreads=3).to_packed()
        monkeypatch.setenv("SFS2D_VCF_HASH_MERGE", "0")
        b = V.read_vcf(path, pm, nthreads=3).to_packed()
        c = V.make_packed_vcf(path, pm, nthreads=3)   # the native pack (scan-ordered files) or its fallback
        for q in (b, c):
            assert np.array_equal(a.counts, q.counts) and np.array_equal(a.pos, q.pos)
            assert np.array_equal(a.chrom_off, q.chrom_off) and a.chrom_names == q.chrom_names
            assert np.array_equal(a.ann_id, q.ann_id) and a.ann_names == q.ann_names
    else:   # int() of the POS text raises in the general path, which the native pack falls back to
        with pytest.raises(ValueError):
            V.read_vcf(path, pm).to_packed()
        with pytest.raises(ValueError):
            V.make_packed_vcf(path, pm)


def test_bgzf_multi_block(tmp_path):
    sys.path.insert(0, GOLD)
    from gen_golden_vcf import bgzf_bytes   # BGZF writer (data only; no reference code)
    raw = synth_vcf(30000, SAMPLES, seed=9)
    path = str(tmp_path / "b.vcf.gz")
    open(path, "wb").write(bgzf_bytes(raw.replace(b"\r\n", b"\n"), block=5000))
    pm = str(tmp_path / "pm.txt")
    write_popmap(pm, [(s, ["uv", "bv"][i % 2]) for i, s in enumerate(SAMPLES)])
    same_dict(V.read_vcf(path, pm, nthreads=8).to_data_dict(), vcf_oracle.make_data_dict_vcf(path, pm))


@pytest.mark.parametrize("bad,exc", [
    ((123, "chr1\t5\t.\tA\tC\t.\tPASS"), IndexError),                      # no INFO column
    ((30000, "chr1\t5\t.\tA\tC\t.\tPASS\tX"), IndexError),                 # no FORMAT column (late chunk)
    ((777, "chr1\t5\t.\tA\tC\t.\tPASS\tX\tDP\t" + "\t".join(["1"] * 24)), ValueError),   # no GT
    ((20001, "chr1\t5\t.\tA\tC\t.\t.\tX\tDP:GT\t" + "\t".join(["1"] * 24)), IndexError),  # GT subfield missing
])
def test_errors_like_reference(tmp_path, bad, exc):
    raw = synth_vcf(40000, SAMPLES, seed=2, bad=bad)
    path = str(tmp_path / "e.vcf")
    open(path, "wb").write(raw)
    pm = str(tmp_path / "pm.txt")
    write_popmap(pm, [(s, "uv") for s in SAMPLES])
    with pytest.raises(exc):
        vcf_oracle.make_data_dict_vcf(path, pm)
    for nt in (1, 8):
        with pytest.raises(exc):
            V.read_vcf(path, pm, nthreads=nt)


def test_filtered_errors_are_not_raised(tmp_path):
    # a FILTER-failing or non-ACGT line never reaches the GT lookup (twoDSFS_class.py:101-109)
    raw = synth_vcf(3000, SAMPLES, seed=3, bad=(10, "chr1\t5\t.\tA\tC\t.\tq10\tX\tDP"))
    path = str(tmp_path / "f.vcf")
    open(path, "wb").write(raw)
    pm = str(tmp_path / "pm.txt")
    write_popmap(pm, [(s, "uv") for s in SAMPLES])
    same_dict(V.read_vcf(path, pm).to_data_dict(), vcf_oracle.make_data_dict_vcf(path, pm))


def test_missing_files(tmp_path):
    with pytest.raises(FileNotFoundError):
        V.read_vcf(str(tmp_path / "nope.vcf.gz"), os.path.join(GOLD, "popmap_ref.txt"))


@pytest.mark.skipif(not os.path.exists("/root/reference/vcf_pruned/ECB_LDprunedv2.vcf.gz"),
                    reason="reference data not present")
def test_full_reference_vcf_digest():
    sys.path.insert(0, GOLD)
    from gen_golden_vcf import digest
    man = json.load(open(os.path.join(GOLD, "vcf_manifest.json")))["full_ECB_LDprunedv2"]
    d = V.make_data_dict_vcf("/root/reference/vcf_pruned/ECB_LDprunedv2.vcf.gz", "/root/reference/popmap.txt")
    assert len(d) == man["records"] and digest(d) == man["digest"]
