"""VCF(.gz / BGZF) + popmap ingest through the native parser (include/sfs2d_ingest.h).

Drop-in for ``make_data_dict_vcf(vcf_filename, popinfo_filename)`` (twoDSFS_class.py:36-138;
sims_scan.py:18-120), with its semantics (quirks Q10/Q12/Q13) -- see the header
for the rules.  ``read_vcf`` returns the parsed columns; from them

* ``VcfTable.to_data_dict()`` rebuilds the reference's dict
  ``{"CHR-POS": {"segregating", "context", "calls", "annotation"}}`` in the same key order, and
* ``VcfTable.to_packed(pop1, pop2)`` goes straight to the packed SoA the HIP kernels stream
  (scan order: chromosome string, then integer position, dict order on ties -- exactly what
  ``pack_snp_dict(make_data_dict_vcf(...))`` gives, without building the dict).

The parser is C++ (``libsfs2d_ingest.so``, built by ``make -C 2dsfs-scan_amd/csrc``); without it
every call raises ``Sfs2dError``.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Sequence

import numpy as np

from ._lib import Sfs2dError
from .pack import PackedSNPs, MAX_COUNT

HERE = os.path.dirname(os.path.abspath(__file__))
INGEST_PATH = os.environ.get("SFS2D_INGEST_LIB", os.path.join(HERE, "..", "csrc", "libsfs2d_ingest.so"))

# exported symbols of include/sfs2d_ingest.h (checked by tests/test_vcf_ingest.py)
EXPORTS = [
    "sfs2d_vcf_read", "sfs2d_vcf_free", "sfs2d_vcf_last_error", "sfs2d_vcf_num_records", "sfs2d_vcf_num_pops",
    "sfs2d_vcf_pop_name", "sfs2d_vcf_num_chroms", "sfs2d_vcf_chrom_name", "sfs2d_vcf_num_annotations",
    "sfs2d_vcf_annotation", "sfs2d_vcf_columns", "sfs2d_vcf_stats", "sfs2d_vcf_pack",
]
E_INDEX, E_VALUE = -3, -4

_ilib = None


def ingest_lib():
    global _ilib
    if _ilib is not None:
        return _ilib
    if not os.path.exists(INGEST_PATH):
        raise Sfs2dError(-1, f"native VCF parser not built: {INGEST_PATH} (make -C 2dsfs-scan_amd/csrc)")
    L = C.CDLL(INGEST_PATH)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    L.sfs2d_vcf_read.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(vp)]
    L.sfs2d_vcf_free.argtypes = [vp]
    L.sfs2d_vcf_last_error.restype = C.c_char_p
    for f in ("sfs2d_vcf_num_pops", "sfs2d_vcf_num_chroms", "sfs2d_vcf_num_annotations"):
        getattr(L, f).argtypes = [vp]
        getattr(L, f).restype = i32
    L.sfs2d_vcf_num_records.argtypes = [vp]
    L.sfs2d_vcf_num_records.restype = i64
    for f in ("sfs2d_vcf_pop_name", "sfs2d_vcf_chrom_name", "sfs2d_vcf_annotation"):
        getattr(L, f).argtypes = [vp, i32]
        getattr(L, f).restype = C.c_char_p
    L.sfs2d_vcf_columns.argtypes = [vp] + [C.POINTER(vp)] * 7
    L.sfs2d_vcf_stats.argtypes = [vp, C.POINTER(i64), C.POINTER(i64)] + [C.POINTER(C.c_double)] * 3
    L.sfs2d_vcf_pack.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, vp, vp]
    _ilib = L
    return L


def _view(ptr, dtype, count):
    if count == 0:
        return np.zeros(0, dtype)
    buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype).copy()


class _PosTexts(Sequence):
    """POS texts of the records, decoded from the library's blob on first use (the packed path reads
    only the numeric positions, so a million-record ingest builds no per-record strings)."""

    def __init__(self, blob: bytes, pos_off: np.ndarray):
        self._blob, self._off, self._list = blob, pos_off, None

    def _all(self) -> List[str]:
        if self._list is None:
            text = self._blob.decode("utf-8", "surrogateescape")
            po = self._off.tolist()
            if len(text) == len(self._blob):   # ASCII: character offsets are byte offsets
                self._list = [text[po[i]:po[i + 1]] for i in range(len(po) - 1)]
            else:
                self._list = [self._blob[po[i]:po[i + 1]].decode("utf-8", "surrogateescape") for i in range(len(po) - 1)]
        return self._list

    def __len__(self):
        return len(self._off) - 1

    def __getitem__(self, i):
        if self._list is None and isinstance(i, int):
            k = i + len(self) if i < 0 else i
            if not 0 <= k < len(self):
                raise IndexError(i)
            return self._blob[int(self._off[k]):int(self._off[k + 1])].decode("utf-8", "surrogateescape")
        return self._all()[i]

    def __iter__(self):
        return iter(self._all())


@dataclass
class VcfTable:
    """Parsed records in dict insertion order (one per distinct CHROM-POS key)."""
    pops: List[str]
    chrom_names: List[str]
    ann_names: List[str]
    chrom: np.ndarray      # int32 [n]
    pos: np.ndarray        # int64 [n]; INT64_MIN where POS is not a plain decimal
    pos_text: List[str]    # POS as written (the key is f"{chrom}-{pos_text}")
    ann: np.ndarray        # int32 [n]
    alleles: np.ndarray    # uint8 [n, 2] upper-case REF / ALT
    calls: np.ndarray      # int32 [n, P, 2]; -1 = population absent from the record
    stats: dict

    @property
    def n(self) -> int:
        return int(len(self.chrom))

    def keys(self) -> List[str]:
        return [f"{self.chrom_names[c]}-{t}" for c, t in zip(self.chrom.tolist(), self.pos_text)]

    def to_data_dict(self) -> dict:
        """The reference's make_data_dict_vcf dict (same keys, order, values and types)."""
        out = {}
        ref = [chr(x) for x in self.alleles[:, 0].tolist()]
        alt = [chr(x) for x in self.alleles[:, 1].tolist()]
        calls = self.calls.tolist()
        anns = [self.ann_names[a] for a in self.ann.tolist()]
        for i, key in enumerate(self.keys()):
            cd = {}
            for j, (r, a) in enumerate(calls[i]):
                if r >= 0:
                    cd[self.pops[j]] = (r, a)
            out[key] = {"segregating": (ref[i], alt[i]), "context": "-" + ref[i] + "-", "calls": cd,
                        "annotation": anns[i]}
        return out

    def to_packed(self, pop1: str = "uv", pop2: str = "bv") -> PackedSNPs:
        """pack_snp_dict(to_data_dict(), pop1, pop2) without the dict (twoDSFS_class.py:828-835 order)."""
        for name in self.chrom_names:
            if "-" in name:
                raise ValueError(f"too many values to unpack in SNP keys of chromosome {name!r}")
        pos = self.pos.copy()
        bad = np.nonzero(pos == np.iinfo(np.int64).min)[0]
        for i in bad.tolist():
            t = self.pos_text[i]
            if "-" in t:
                raise ValueError(f"too many values to unpack in SNP key {self.chrom_names[self.chrom[i]]}-{t}")
            pos[i] = int(t)   # ValueError for non-numbers, as int() in the reference's sort key
        if pos.size and (pos.min() < 0 or pos.max() > 0xFFFFFFFF):
            raise ValueError("positions must fit in uint32")
        rank = np.empty(len(self.chrom_names), np.int64)
        order_names = sorted(range(len(self.chrom_names)), key=lambda c: self.chrom_names[c])
        rank[order_names] = np.arange(len(order_names))
        crank = rank[self.chrom] if self.n else np.zeros(0, np.int64)
        # a file already in (chromosome name, position) order (the common case) keeps its order:
        # the stable sort would return the identity
        dc = np.diff(crank)
        if self.n and bool(np.all((dc > 0) | ((dc == 0) & (np.diff(pos) >= 0)))):
            order = slice(None)
        else:
            order = np.lexsort((pos, crank))      # stable: dict order among equal (chrom, pos)
        crank_s = crank[order]

        calls = self.calls if isinstance(order, slice) else self.calls[order]

        def pop_counts(pop):
            """(ref, alt) of pop per record as uint32: calls.get(pop, (0, 0))"""
            if pop not in self.pops:
                z = np.zeros(self.n, np.uint32)
                return z, z
            c = np.maximum(calls[:, self.pops.index(pop), :], 0)
            if c.size and int(c.max()) > MAX_COUNT:
                raise ValueError("allele counts above 255 do not fit the packed u8x4 layout")
            c = c.astype(np.uint32)
            return c[:, 0], c[:, 1]
        r1, a1 = pop_counts(pop1)
        r2, a2 = pop_counts(pop2)
        counts = r1 | (a1 << 8) | (r2 << 16) | (a2 << 24)
        bounds = np.nonzero(np.diff(crank_s))[0] + 1 if self.n else np.zeros(0, np.int64)
        offs = np.concatenate([[0], bounds, [self.n]]).astype(np.int64) if self.n else np.zeros(1, np.int64)
        names = [self.chrom_names[order_names[int(r)]] for r in crank_s[offs[:-1]]] if self.n else []
        if len(self.ann_names) > 65535:
            raise ValueError("more than 65535 distinct annotations")
        return PackedSNPs(counts, pos[order].astype(np.uint32), offs, names,
                          self.ann[order].astype(np.uint16), list(self.ann_names), pop1, pop2)


def _open(vcf_filename, popinfo_filename, nthreads):
    """The native parse; raises the reference's exception types.  Returns the library's handle."""
    L = ingest_lib()
    h = C.c_void_p()
    rc = L.sfs2d_vcf_read(os.fsencode(str(vcf_filename)), os.fsencode(str(popinfo_filename)), int(nthreads),
                          C.byref(h))
    if rc != 0:
        msg = (L.sfs2d_vcf_last_error() or b"").decode(errors="replace")
        if rc == E_INDEX:
            raise IndexError(msg)
        if rc == E_VALUE:
            raise ValueError(msg)
        if rc == -1:
            raise FileNotFoundError(msg)
        raise Sfs2dError(rc, msg)
    return L, h


def _names(L, h):
    dec = (lambda b: b.decode("utf-8", "surrogateescape"))
    pops = [dec(L.sfs2d_vcf_pop_name(h, i)) for i in range(int(L.sfs2d_vcf_num_pops(h)))]
    chroms = [dec(L.sfs2d_vcf_chrom_name(h, i)) for i in range(L.sfs2d_vcf_num_chroms(h))]
    anns = [dec(L.sfs2d_vcf_annotation(h, i)) for i in range(L.sfs2d_vcf_num_annotations(h))]
    return pops, chroms, anns


def _table(L, h) -> VcfTable:
    n = int(L.sfs2d_vcf_num_records(h))
    pops, chroms, anns = _names(L, h)
    P = len(pops)
    ptrs = [C.c_void_p() for _ in range(7)]
    L.sfs2d_vcf_columns(h, *[C.byref(p) for p in ptrs])
    chrom = _view(ptrs[0].value, np.int32, n)
    pos = _view(ptrs[1].value, np.int64, n)
    pos_off = _view(ptrs[3].value, np.int64, n + 1)
    blob = C.string_at(ptrs[2].value, int(pos_off[-1])) if n and pos_off[-1] else b""
    texts = _PosTexts(blob, pos_off)
    ann = _view(ptrs[4].value, np.int32, n)
    alle = _view(ptrs[5].value, np.uint8, 2 * n).reshape(n, 2)
    calls = _view(ptrs[6].value, np.int32, n * P * 2).reshape(n, P, 2)
    tb, ln = C.c_int64(), C.c_int64()
    t = [C.c_double() for _ in range(3)]
    L.sfs2d_vcf_stats(h, C.byref(tb), C.byref(ln), *[C.byref(x) for x in t])
    stats = {"text_bytes": tb.value, "lines": ln.value, "t_inflate": t[0].value, "t_parse": t[1].value,
             "t_merge": t[2].value}
    return VcfTable(pops, chroms, anns, chrom, pos, texts, ann, alle, calls, stats)


def read_vcf(vcf_filename, popinfo_filename, nthreads: int = 0) -> VcfTable:
    """Parse with the native multithreaded parser; raises the reference's exception types."""
    L, h = _open(vcf_filename, popinfo_filename, nthreads)
    try:
        return _table(L, h)
    finally:
        L.sfs2d_vcf_free(h)


def _packed_fast(L, h, pop1, pop2):
    """VcfTable.to_packed for a file already in scan order, packed natively (sfs2d_vcf_pack) from the
    library's table without copying its columns; None when that path does not apply."""
    n = int(L.sfs2d_vcf_num_records(h))
    pops, chroms, anns = _names(L, h)
    if n == 0 or any("-" in c for c in chroms):
        return None
    order_names = sorted(range(len(chroms)), key=lambda c: chroms[c])
    rank = np.empty(len(chroms), np.int32)
    rank[order_names] = np.arange(len(order_names), dtype=np.int32)
    counts = np.empty(n, np.uint32)
    pos = np.empty(n, np.uint32)
    ann = np.empty(n, np.uint16)
    i1 = pops.index(pop1) if pop1 in pops else -1
    i2 = pops.index(pop2) if pop2 in pops else -1
    rc = L.sfs2d_vcf_pack(h, rank.ctypes.data, i1, i2, counts.ctypes.data, pos.ctypes.data, ann.ctypes.data)
    if rc != 0:
        return None
    ptrs = [C.c_void_p() for _ in range(7)]
    L.sfs2d_vcf_columns(h, *[C.byref(p) for p in ptrs])
    chrom = np.frombuffer((C.c_char * (4 * n)).from_address(ptrs[0].value), dtype=np.int32)   # borrowed
    crank = rank[chrom]
    bounds = np.nonzero(np.diff(crank))[0] + 1
    offs = np.concatenate([[0], bounds, [n]]).astype(np.int64)
    names = [chroms[order_names[int(r)]] for r in crank[offs[:-1]]]
    return PackedSNPs(counts, pos, offs, names, ann, list(anns), pop1, pop2)


def make_data_dict_vcf(vcf_filename, popinfo_filename):
    """twoDSFS_class.py:36-138 / sims_scan.py:18-120: the reference's SNP dict."""
    return read_vcf(vcf_filename, popinfo_filename).to_data_dict()


def make_packed_vcf(vcf_filename, popinfo_filename, pop1: str = "uv", pop2: str = "bv",
                    nthreads: int = 0) -> PackedSNPs:
    """VCF + popmap straight to the packed scan-order arrays (no dict): natively for a file in scan
    order, else through VcfTable.to_packed (which also raises the reference's errors)."""
    L, h = _open(vcf_filename, popinfo_filename, nthreads)
    try:
        p = _packed_fast(L, h, pop1, pop2)
        tab = None if p is not None else _table(L, h)
    finally:
        L.sfs2d_vcf_free(h)
    return p if p is not None else tab.to_packed(pop1, pop2)
