"""Packed SNP layout (struct-of-arrays) that the HIP kernels stream from HBM.

The reference keeps SNPs as a dict ``{"CHR-POS": {"calls": {pop: (ref, alt)},
"annotation": str, ...}}`` (twoDSFS_class.py:90-134) and re-walks it, splitting
the key string, inside every window (twoDSFS_class.py:176, 415, 828-835).
Here the dict is packed once, in the reference's scan order -- chromosome accession
in Python string order, then integer position (twoDSFS_class.py:828-835, quirk Q10) --
into:

* ``counts``  uint32[n]: bytes (ref1, alt1, ref2, alt2), little-endian, i.e.
  ``ref1 | alt1<<8 | ref2<<16 | alt2<<24`` (4 B/SNP, one coalesced dword per lane);
* ``pos``     uint32[n]: 1-based position (4 B/SNP);
* ``ann_id``  uint16[n]: index into ``ann_names`` (only read when a variant_type
  filter is active; turned into a 1-byte mask at scan time);
* ``chrom_off`` int64[nchrom+1]: CSR offsets of each chromosome's SNP run.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

__all__ = ["PackedSNPs", "pack_snp_dict", "to_snp_dict", "pack_counts"]

MAX_COUNT = 255  # u8 per allele count: 2*pop_size must be <= 255


def pack_counts(r1, a1, r2, a2) -> np.ndarray:
    r1 = np.asarray(r1, dtype=np.uint32)
    a1 = np.asarray(a1, dtype=np.uint32)
    r2 = np.asarray(r2, dtype=np.uint32)
    a2 = np.asarray(a2, dtype=np.uint32)
    if max(int(r1.max(initial=0)), int(a1.max(initial=0)), int(r2.max(initial=0)),
           int(a2.max(initial=0))) > MAX_COUNT:
        raise ValueError("allele counts above 255 do not fit the packed u8x4 layout")
    return (r1 | (a1 << 8) | (r2 << 16) | (a2 << 24)).astype(np.uint32)


@dataclass
class PackedSNPs:
    counts: np.ndarray
    pos: np.ndarray
    chrom_off: np.ndarray
    chrom_names: List[str]
    ann_id: np.ndarray
    ann_names: List[str] = field(default_factory=list)
    pop1: str = "uv"
    pop2: str = "bv"

    def __post_init__(self):
        self.counts = np.ascontiguousarray(self.counts, dtype=np.uint32)
        self.pos = np.ascontiguousarray(self.pos, dtype=np.uint32)
        self.chrom_off = np.ascontiguousarray(self.chrom_off, dtype=np.int64)
        if self.ann_id is None:
            self.ann_id = np.zeros(len(self.counts), dtype=np.uint16)
        self.ann_id = np.ascontiguousarray(self.ann_id, dtype=np.uint16)
        if len(self.counts) != len(self.pos) or len(self.counts) != len(self.ann_id):
            raise ValueError("counts/pos/ann_id length mismatch")
        if len(self.chrom_off) != len(self.chrom_names) + 1:
            raise ValueError("chrom_off must have nchrom+1 entries")
        if len(self.chrom_off) and (self.chrom_off[0] != 0 or self.chrom_off[-1] != len(self.counts)):
            raise ValueError("chrom_off must start at 0 and end at n")

    @property
    def n(self) -> int:
        return int(len(self.counts))

    @property
    def nchrom(self) -> int:
        return len(self.chrom_names)

    def field(self, shift: int) -> np.ndarray:
        return ((self.counts >> np.uint32(shift)) & np.uint32(0xFF)).astype(np.int64)

    @property
    def ref1(self):
        return self.field(0)

    @property
    def alt1(self):
        return self.field(8)

    @property
    def ref2(self):
        return self.field(16)

    @property
    def alt2(self):
        return self.field(24)

    def chrom_of(self) -> np.ndarray:
        """Chromosome index of every SNP."""
        return np.repeat(np.arange(self.nchrom, dtype=np.int64), np.diff(self.chrom_off))

    def variant_mask(self, variant_type: Optional[str]) -> Optional[np.ndarray]:
        """1 where the SNP's annotation equals ``variant_type`` (None = no filter).

        Mirrors ``snp_info.get('annotation') != variant_type`` (twoDSFS_class.py:185-187)
        and ``count_snps`` (291-302)."""
        if variant_type is None:
            return None
        try:
            want = self.ann_names.index(variant_type)
        except ValueError:
            return np.zeros(self.n, dtype=np.uint8)
        return (self.ann_id == want).astype(np.uint8)

    def single_pop(self, pop: str) -> "PackedSNPs":
        """Both count slots set to population ``pop`` ((0, 0) when absent: calls.get(pop, (0, 0)))."""
        if pop == self.pop1:
            lo = self.counts & np.uint32(0xFFFF)
        elif pop == self.pop2:
            lo = self.counts >> np.uint32(16)
        else:
            lo = np.zeros_like(self.counts)
        return PackedSNPs(lo | (lo << np.uint32(16)), self.pos, self.chrom_off, list(self.chrom_names),
                          self.ann_id, list(self.ann_names), pop, pop)

    def slice_snps(self, lo: int, hi: int):
        """(SNPs [lo, hi) of the scan order as a data set of the chromosomes they touch, index of its
        first chromosome here): a rank's part of a data set split at window boundaries (sfs2d.dist)."""
        if hi <= lo:
            return PackedSNPs(self.counts[:0], self.pos[:0], np.zeros(1, np.int64), [], self.ann_id[:0],
                              list(self.ann_names), self.pop1, self.pop2), 0
        c0 = int(np.searchsorted(self.chrom_off, lo, side="right")) - 1
        c1 = int(np.searchsorted(self.chrom_off, hi, side="left"))      # chromosomes c0 .. c1-1
        off = np.clip(self.chrom_off[c0:c1 + 1], lo, hi) - lo
        return PackedSNPs(self.counts[lo:hi], self.pos[lo:hi], off, list(self.chrom_names[c0:c1]),
                          self.ann_id[lo:hi], list(self.ann_names), self.pop1, self.pop2), c0

    def subset_chroms(self, idx) -> "PackedSNPs":
        idx = list(idx)
        parts_c, parts_p, parts_a, offs = [], [], [], [0]
        for c in idx:
            s, e = int(self.chrom_off[c]), int(self.chrom_off[c + 1])
            parts_c.append(self.counts[s:e])
            parts_p.append(self.pos[s:e])
            parts_a.append(self.ann_id[s:e])
            offs.append(offs[-1] + e - s)
        cat = (lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt))
        return PackedSNPs(cat(parts_c, np.uint32), cat(parts_p, np.uint32), np.array(offs, np.int64),
                          [self.chrom_names[c] for c in idx], cat(parts_a, np.uint16),
                          list(self.ann_names), self.pop1, self.pop2)


def last_key_index(data, p: PackedSNPs) -> int:
    """Index in ``p`` (scan order) of the data dict's last-inserted key; for packed input the dict
    is the one ``to_snp_dict`` would build (insertion in scan order), i.e. the last SNP."""
    if isinstance(data, PackedSNPs) or p.n == 0:
        return p.n - 1
    key = next(reversed(data))
    chrom, pos = key.split("-")
    c = p.chrom_names.index(chrom)
    lo, hi = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
    return lo + int(np.searchsorted(p.pos[lo:hi], int(pos)))


def shadow_chrom_starts(p: PackedSNPs, last: int, ws: int, start_position=None, end_position=None) -> PackedSNPs:
    """The SNP stream ``T2D_scan`` (twoDSFS_class.py:686-776) actually scores.

    At every chromosome change the driver computes a per-chromosome background with
    ``for snp_key, snp_data in data_dict.items()`` (:740), which rebinds the outer loop's
    ``snp_key``: the chromosome's first SNP then enters its window as the data dict's LAST key
    (its calls and annotation, :748 / :763), while the window itself still follows the first SNP's
    own position (``pos``).  When that last SNP lies in the same window, both are one dict key and
    the window holds it once.  The position filter (:179-182) reads the key's position, so it is
    applied here: filtered SNPs keep their place with (0, 0) counts, which the 2D SFS skips
    (:212-213) and count_snps still counts (:291-302); the scan then runs without it."""
    n = p.n
    counts = p.counts.copy()
    ann = p.ann_id.copy()
    keypos = p.pos.astype(np.int64)
    keep = np.ones(n, dtype=bool)
    if n:
        lc = int(np.searchsorted(p.chrom_off, last, side="right")) - 1
        wid = lambda q: max(int(q) - 1, 0) // int(ws)   # window of a position: start 1 + k ws (:747, :762)
        for c in range(p.nchrom):
            x = int(p.chrom_off[c])
            if x == int(p.chrom_off[c + 1]) or x == last:
                continue
            counts[x] = p.counts[last]
            ann[x] = p.ann_id[last]
            keypos[x] = int(p.pos[last])
            if c == lc and wid(p.pos[x]) == wid(p.pos[last]):
                keep[x] = False
    drop = np.zeros(n, dtype=bool)
    if start_position is not None:
        drop |= keypos < int(start_position)
    if end_position is not None:
        drop |= keypos > int(end_position)
    counts[drop] = 0
    if keep.all():
        return PackedSNPs(counts, p.pos, p.chrom_off, list(p.chrom_names), ann, list(p.ann_names), p.pop1, p.pop2)
    cum = np.concatenate([[0], np.cumsum(keep)])
    off = cum[p.chrom_off]
    return PackedSNPs(counts[keep], p.pos[keep], off, list(p.chrom_names), ann[keep], list(p.ann_names),
                      p.pop1, p.pop2)


def pack_snp_dict(data_dict: dict, pop1: str = "uv", pop2: str = "bv") -> PackedSNPs:
    """Pack the reference SNP dict into scan order.

    Missing populations count as (0, 0) exactly like ``snp_info['calls'].get(pop, (0, 0))``
    (twoDSFS_class.py:190-191).  Keys are split on the first '-' like ``snp_id.split('-')``
    (a second '-' in the key makes the reference raise ValueError; so do we)."""
    rows = []
    for key, info in data_dict.items():
        parts = key.split("-")
        if len(parts) != 2:
            raise ValueError(f"too many values to unpack in SNP key {key!r}")
        rows.append((parts[0], int(parts[1]), key))
    rows.sort(key=lambda x: (x[0], x[1]))
    n = len(rows)
    r1 = np.zeros(n, np.int64)
    a1 = np.zeros(n, np.int64)
    r2 = np.zeros(n, np.int64)
    a2 = np.zeros(n, np.int64)
    pos = np.zeros(n, np.int64)
    ann = np.zeros(n, np.int64)
    ann_names: List[str] = []
    ann_index = {}
    chrom_names: List[str] = []
    offs = [0]
    prev = None
    for i, (chrom, p, key) in enumerate(rows):
        if chrom != prev:
            if prev is not None:
                offs.append(i)
            chrom_names.append(chrom)
            prev = chrom
        info = data_dict[key]
        calls = info["calls"]
        c1 = calls.get(pop1, (0, 0))
        c2 = calls.get(pop2, (0, 0))
        r1[i], a1[i] = c1[0], c1[1]
        r2[i], a2[i] = c2[0], c2[1]
        pos[i] = p
        a = info.get("annotation")
        j = ann_index.get(a)
        if j is None:
            j = len(ann_names)
            ann_index[a] = j
            ann_names.append(a)
        ann[i] = j
    offs.append(n)
    if n == 0:
        offs = [0]
    if pos.size and (pos.min() < 0 or pos.max() > 0xFFFFFFFF):
        raise ValueError("positions must fit in uint32")
    if len(ann_names) > 65535:
        raise ValueError("more than 65535 distinct annotations")
    return PackedSNPs(pack_counts(r1, a1, r2, a2), pos.astype(np.uint32), np.array(offs, np.int64),
                      chrom_names, ann.astype(np.uint16), [str(x) if x is not None else "" for x in ann_names],
                      pop1, pop2)


def to_snp_dict(p: PackedSNPs) -> dict:
    """Inverse of pack_snp_dict: rebuild the reference's dict (test fixture generation)."""
    out = {}
    r1, a1, r2, a2 = p.ref1, p.alt1, p.ref2, p.alt2
    chrom = p.chrom_of()
    for i in range(p.n):
        key = f"{p.chrom_names[chrom[i]]}-{int(p.pos[i])}"
        out[key] = {
            "calls": {p.pop1: (int(r1[i]), int(a1[i])), p.pop2: (int(r2[i]), int(a2[i]))},
            "annotation": p.ann_names[int(p.ann_id[i])] if p.ann_names else "No annotation",
        }
    return out
