"""Drop-in replacement for the reference module ``scripts/src/twoDSFS_class.py``.

Same class, method names, arguments, return shapes and error behaviour as the reference's
``LikelihoodInference_jointSFS`` (twoDSFS_class.py:20-1737) for the window-scan path, plus the
module-level ``col_names`` / ``chr_ids`` / ``save_csv_stats`` CSV writer (1788-1797, 1881-1907).
Every window statistic is computed by the HIP kernels of ``csrc/sfs2d.hip`` on an MI355X
(through ``sfs2d.engine``); there is no CPU fallback.

Methods accept either the reference's SNP dict (``{"CHR-POS": {"calls": ..., "annotation": ...}}``)
or an already packed ``sfs2d.PackedSNPs`` (skips the dict packing, which dominates host time).
"""
from __future__ import annotations

import csv
import os
from typing import Optional

import numpy as np

from sfs2d import _lib as L
from sfs2d import post
from sfs2d.engine import Engine, ScanConfig
from sfs2d.vcf import make_data_dict_vcf as _make_data_dict_vcf
from sfs2d.pack import PackedSNPs, last_key_index, pack_snp_dict, shadow_chrom_starts

__all__ = ["LikelihoodInference_jointSFS", "save_csv_stats", "col_names", "chr_ids", "load_chr_ids"]

_NO_ANN = 1 << 20   # an annotation id no SNP carries (variant_type absent from the data)

col_names = ['chromosome', 'window_start', 'window_end', 'snp_count', 'T2D', 'T1D_p1', 'T1D_p2',
             'new_term_p1', 'new_term_p2', 'T2D_diff']
chr_ids: dict = {}


def load_chr_ids(path: str) -> dict:
    """Accession -> chromosome number map (chromosomes.txt; reference 1788-1797)."""
    chr_ids.clear()
    with open(path, "r") as fh:
        for line in fh:
            columns = line.strip().split("\t")
            if len(columns) >= 2:
                chr_ids[columns[0]] = columns[1]
    return chr_ids


if os.environ.get("SFS2D_CHROMOSOMES"):
    load_chr_ids(os.environ["SFS2D_CHROMOSOMES"])


def save_csv_stats(stats_dict, output):
    """twoDSFS_class.py:1884-1907: one row per window, chromosome renamed through chr_ids."""
    with open(output, 'w', newline='') as csvfile:
        writer = csv.DictWriter(csvfile, fieldnames=col_names)
        writer.writeheader()
        for window_coords, result in stats_dict.items():
            chromosome = window_coords.split(' ')[0]
            chromosome_num = chr_ids.get(chromosome, chromosome)
            window_start, window_end = window_coords.split(' ')[1].split('-')
            writer.writerow({
                'chromosome': chromosome_num, 'window_start': window_start, 'window_end': window_end,
                'snp_count': result["snp_count"], 'T2D': result["T2D"], 'T1D_p1': result["T1D_pop1"],
                'T1D_p2': result["T1D_pop2"], 'new_term_p1': result["new_term_pop1"],
                'new_term_p2': result["new_term_pop2"], 'T2D_diff': result["T2D_diff"]})


def _fold_counts(u: np.ndarray) -> np.ndarray:
    """fold_1d_sfs on a dense unfolded spectrum: folded[f] = u[f] + u[2n-f], folded[n] = u[n]."""
    n2 = len(u) - 1
    n = n2 // 2
    out = np.zeros(n + 1, dtype=u.dtype)
    for f in range(n2 + 1):
        out[min(f, n2 - f)] += u[f]
    return out


class LikelihoodInference_jointSFS:
    def __init__(self, vcf_filename, popinfo_filename, start_position=None, end_position=None,
                 pop1='uv', pop2='bv', pop1_size=18, pop2_size=14, variant_type=None, fold=True, device=0,
                 distributed=False):
        """The reference's constructor (twoDSFS_class.py:21-33), plus ``device`` (the GPU of this
        process) and ``distributed``: with a torch.distributed process group (one process per GPU),
        every window scan is split over the group at window boundaries balanced by SNPs -- one
        chromosome spread over several ranks, its background histograms all-reduced -- and every rank
        returns the whole result (sfs2d.dist.scan_records_split); ``distributed="chromosomes"`` shards
        whole chromosomes instead (no collective before the scan; sfs2d.dist.scan_records).  All
        ranks must make the same calls."""
        self.vcf_filename = vcf_filename
        self.popinfo_filename = popinfo_filename
        self.pop1 = pop1
        self.pop2 = pop2
        self.pop1_size = pop1_size
        self.pop2_size = pop2_size
        self.start_position = start_position
        self.end_position = end_position
        self.variant_type = variant_type
        self.fold = fold
        self.device = device
        self.distributed = distributed

    # ------------------------------------------------------------------ ingest
    def make_data_dict_vcf(self, vcf_filename=None, popinfo_filename=None):
        """twoDSFS_class.py:36-138 (quirks Q12/Q13 kept; see sfs2d.vcf)."""
        return _make_data_dict_vcf(vcf_filename if vcf_filename is not None else self.vcf_filename,
                                   popinfo_filename if popinfo_filename is not None else self.popinfo_filename)

    # ------------------------------------------------------------------ plumbing
    def _engine(self) -> Engine:
        return Engine.get(self.device)

    def _pack(self, data, pop1=None, pop2=None) -> PackedSNPs:
        if isinstance(data, PackedSNPs):
            return data
        return pack_snp_dict(data, pop1 or self.pop1, pop2 or self.pop2)

    def _cfg(self, p: PackedSNPs, **kw) -> ScanConfig:
        ann = -1
        if self.variant_type is not None:
            ann = p.ann_names.index(self.variant_type) if self.variant_type in p.ann_names else _NO_ANN
        start = None if self.start_position is None else int(self.start_position)
        end = None if self.end_position is None else int(self.end_position)
        return ScanConfig(n1p=self.pop1_size, n2p=self.pop2_size, fold=bool(self.fold), ann_want=ann,
                          start_position=start, end_position=end, **kw)

    def _scan(self, p: PackedSNPs, cfg: ScanConfig, bg=None):
        if self.distributed:
            from sfs2d import dist as D
            if self.distributed == "chromosomes":
                return D.scan_records(p, cfg, bg, self._scan_local, self.device)
            return D.scan_records_split(p, cfg, bg, self._split_scan, self.device)
        return self._scan_local(p, cfg, bg)

    def _split_scan(self, p: PackedSNPs, cfg: ScanConfig, bg=None):
        from sfs2d.engine import SplitJob
        return SplitJob(self._engine(), p, cfg, bg)
    _split_scan.device_rows = True   # its jobs exchange background rows in HBM (sfs2d.dist._split_device)

    def _hist(self, p: PackedSNPs, cfg: ScanConfig, chrom: int):
        """Background histograms (h2d, unfolded h1a, unfolded h1b) of chromosome ``chrom`` (-1: all
        SNPs) on the GPU; distributed: every rank histograms a slice, one all-reduce on the device
        (sfs2d.dist.sharded_bg_hist)."""
        if self.distributed:
            from sfs2d import dist as D
            return D.sharded_bg_hist(p, cfg, self.device, chrom)
        eng = self._engine()
        dev = eng.upload(p if chrom < 0 else p.subset_chroms([chrom]))
        try:
            return eng.bg_hist(dev, cfg, -1)
        finally:
            dev.close()

    def _scan_local(self, p: PackedSNPs, cfg: ScanConfig, bg=None):
        eng = self._engine()
        dev = eng.upload(p)
        try:
            recs = eng.scan(dev, cfg, bg)
        finally:
            dev.close()
        return recs

    def _bg_arrays(self, p: PackedSNPs, chrom: int):
        """Unnormalised background of one chromosome (2D grid + folded 1D), computed on the GPU
        (distributed: sharded over the ranks, one all-reduce)."""
        h2, u1, u2 = self._hist(p, self._cfg(p), chrom)
        return h2, _fold_counts(u1), _fold_counts(u2)

    # ------------------------------------------------------------------ window scans
    def combined_scan(self, data_dict, window_size):
        """Each chromosome is its own background (twoDSFS_class.py:787-991)."""
        self.data_dict = data_dict
        self.window_size = window_size
        p = self._pack(data_dict)
        recs = self._scan(p, self._cfg(p, window_mode=L.WINDOW_BP, window=window_size,
                                       bg_mode=L.BG_PER_CHROM, prev_extra=True))
        return post.combined_scan(recs, p, window_size, post.num_slots(recs))

    def scan_chooseChr(self, data_dict, window_size, background_chromosome):
        """One named chromosome as the background for every window (993-1159)."""
        self.data_dict = data_dict
        self.window_size = window_size
        p = self._pack(data_dict)
        if background_chromosome not in p.chrom_names:
            raise ValueError(f"Background chromosome {background_chromosome} not found in the data.")
        bg = self._bg_arrays(p, p.chrom_names.index(background_chromosome))
        recs = self._scan(p, self._cfg(p, window_mode=L.WINDOW_BP, window=window_size,
                                       bg_mode=L.BG_SUPPLIED), bg)
        return post.fixed_bg_scan(recs, p, window_size, post.num_slots(recs))

    def scan_precomputed_BG(self, data_dict, window_size, bg_2d_sfs, bg_1d_sfs_pop1, bg_1d_sfs_pop2):
        """Caller-supplied (normalised or not) background SFS dicts (1161-1299)."""
        self.data_dict = data_dict
        self.window_size = window_size
        p = self._pack(data_dict)
        bg = (self._bg2d_array(bg_2d_sfs), self._bg1d_array(bg_1d_sfs_pop1, self.pop1_size),
              self._bg1d_array(bg_1d_sfs_pop2, self.pop2_size))
        recs = self._scan(p, self._cfg(p, window_mode=L.WINDOW_BP, window=window_size,
                                       bg_mode=L.BG_SUPPLIED), bg)
        return post.fixed_bg_scan(recs, p, window_size, post.num_slots(recs))

    def scan_chooseChr_bySNPs(self, data_dict, snp_window_size, background_chromosome):
        """Fixed-SNP windows against one named chromosome's NORMALISED background (1303-1420)."""
        self.data_dict = data_dict
        self.snp_window_size = snp_window_size
        p = self._pack(data_dict)
        if background_chromosome not in p.chrom_names:
            raise ValueError(f"Background chromosome {background_chromosome} not found in the data.")
        h2, f1, f2 = self._bg_arrays(p, p.chrom_names.index(background_chromosome))
        bg = (np.array(self._normalize_values(h2.ravel().tolist())),
              np.array(self._normalize_values(f1.tolist())), np.array(self._normalize_values(f2.tolist())))
        recs = self._scan(p, self._cfg(p, window_mode=L.WINDOW_SNPS, window=snp_window_size,
                                       bg_mode=L.BG_SUPPLIED), bg)
        return post.bysnp_scan(recs, p, snp_window_size, with_diff=False, final_warning=True)

    def scan_perChr_bySNPs(self, data_dict, snp_window_size):
        """Fixed-SNP windows, each chromosome its own background (1422-1541)."""
        self.data_dict = data_dict
        self.num_snps = snp_window_size
        p = self._pack(data_dict)
        recs = self._scan(p, self._cfg(p, window_mode=L.WINDOW_SNPS, window=snp_window_size,
                                       bg_mode=L.BG_PER_CHROM))
        return post.bysnp_scan(recs, p, snp_window_size, with_diff=True, final_warning=False)

    # ------------------------------------------------------------------ single-statistic scans
    def _filters(self, p: PackedSNPs):
        ann = -1
        if self.variant_type is not None:
            ann = p.ann_names.index(self.variant_type) if self.variant_type in p.ann_names else _NO_ANN
        return ann

    def T1D_scan(self, data_dict, background_sfs, window_size, pop, pop_size):
        """T1D of population ``pop`` (``pop_size`` individuals) per fixed-bp window against a supplied
        folded 1D background (twoDSFS_class.py:539-623): raw alt counts of ``pop`` (no joint fold),
        folded against 2*pop_size (:576-578), the constructor's position / variant_type filters.
        Returns {label: {"snp_count", "T1D"}}; T1D None for an empty window or background."""
        self.data_dict = data_dict
        self.background_sfs = background_sfs
        self.window_size = window_size
        self.pop = pop
        self.pop_size = pop_size
        p = self._pack(data_dict, pop1=pop, pop2=pop).single_pop(pop)
        if p.n == 0:
            return {}
        n = 2 * int(pop_size)
        # pop in both count slots, no fold: the 2D key (alt, alt) is in the grid exactly when the 1D
        # key is; the 2D statistic (against a dummy background) is not read
        cfg = ScanConfig(n1p=pop_size, n2p=pop_size, fold=False, ann_want=self._filters(p),
                         start_position=None if self.start_position is None else int(self.start_position),
                         end_position=None if self.end_position is None else int(self.end_position),
                         window_mode=L.WINDOW_BP, window=window_size, bg_mode=L.BG_SUPPLIED)
        bg = (np.ones((n + 1) * (n + 1)), self._bg1d_array(background_sfs, pop_size), np.ones(pop_size + 1))
        recs = self._scan(p, cfg, bg)
        return post.single_stat_scan(recs, p, window_size, post.num_slots(recs), 1, "T1D")

    def T2D_scan(self, data_dict, background_2d_sfs, window_size):
        """T2D per fixed-bp window against the SUPPLIED background (twoDSFS_class.py:686-776).  The
        per-chromosome background the reference computes at each chromosome change (:738-744) is not
        used for scoring (:753, :768 read ``self.background_2d_sfs``), but its loop rebinds the SNP key:
        the stream is rebuilt accordingly (``sfs2d.pack.shadow_chrom_starts``).
        Returns {label: {"snp_count", "T2D"}}; T2D None for an empty window or background."""
        self.data_dict = data_dict
        self.background_2d_sfs = background_2d_sfs
        self.window_size = window_size
        p = self._pack(data_dict)
        if p.n == 0:
            return {}
        q = shadow_chrom_starts(p, last_key_index(data_dict, p), window_size, self.start_position, self.end_position)
        cfg = ScanConfig(n1p=self.pop1_size, n2p=self.pop2_size, fold=bool(self.fold), ann_want=self._filters(q),
                         window_mode=L.WINDOW_BP, window=window_size, bg_mode=L.BG_SUPPLIED)
        bg = (self._bg2d_array(background_2d_sfs), np.ones(self.pop1_size + 1), np.ones(self.pop2_size + 1))
        recs = self._scan(q, cfg, bg)
        return post.single_stat_scan(recs, q, window_size, post.num_slots(recs), 2, "T2D")

    # ------------------------------------------------------------------ multi-resolution (extension)
    def multi_scan(self, data_dict, window_sizes=(), snp_window_sizes=(), fst=False):
        """combined_scan at every size in ``window_sizes`` and scan_perChr_bySNPs at every size in
        ``snp_window_sizes`` from ONE pass over the SNP stream (the reference script runs these
        scans one after another over the same data, twoDSFS_class.py:1923-2032): the smallest
        fixed-bp scan is the base plan, the others are attached to it (sfs2d_plan_attach).
        Returns {ws: combined_scan result, "<S>snps": scan_perChr_bySNPs result}, plus
        {"fst": {ws: window_fst result}} when ``fst`` (fixed-bp windows only)."""
        p = self._pack(data_dict)
        bps = sorted(set(int(w) for w in window_sizes))
        snps = [int(x) for x in dict.fromkeys(snp_window_sizes)]
        if not bps and not snps:
            return {}
        specs = [("bp", w) for w in bps] + [("snps", S) for S in snps]
        base_ws = bps[0] if bps else None

        def cfg_of(kind, w):
            bp = kind == "bp"
            want_fst = fst and bp and base_ws is not None   # (the library refuses what it cannot attach)
            return self._cfg(p, window_mode=L.WINDOW_BP if bp else L.WINDOW_SNPS, window=w,
                             bg_mode=L.BG_PER_CHROM, prev_extra=bp, fst=want_fst)
        eng = self._engine()
        dev = eng.upload(p)
        out = {}
        try:
            base = eng.plan(dev, cfg_of(*specs[0]))
            try:
                plans = [base]
                for sp in specs[1:]:
                    c = cfg_of(*sp)
                    try:
                        plans.append(base.attach(c))
                    except L.Sfs2dError:
                        if not c.fst:
                            raise
                        c.fst = False   # Fst for this window size from its own plan below
                        plans.append(base.attach(c))
                base.run()
                base.check()
                for (kind, w), pl in zip(specs, plans):
                    pl.check()
                    recs = pl.read()
                    if kind == "bp":
                        out[w] = post.combined_scan(recs, p, w, post.num_slots(recs))
                        if pl.cfg.fst:
                            out.setdefault("fst", {})[w] = post.window_fst_labels(recs, pl.read_fst(), p, w, True)
                    else:
                        out[f"{w}snps"] = post.bysnp_scan(recs, p, w, with_diff=True, final_warning=False)
            finally:
                base.close()
        finally:
            dev.close()
        if fst:
            for w in bps:
                if w not in out.get("fst", {}):
                    out.setdefault("fst", {})[w] = self.window_fst(p, window_size=w)
        return out

    # ------------------------------------------------------------------ Fst (extension)
    def window_fst(self, data_dict, window_size=None, snp_window_size=None):
        """Hudson's Fst per window (not in the reference, whose published FST column is pixy's
        Weir-Cockerham joined in R, ECBstats_plots.R:16-41): {label: Fst or None}, labels as
        combined_scan (fixed bp, ``window_size``) or scan_perChr_bySNPs (``snp_window_size``) emit
        them.  Computed by k_prep on the GPU ("Fst")."""
        p = self._pack(data_dict)
        if (window_size is None) == (snp_window_size is None):
            raise ValueError("give exactly one of window_size / snp_window_size")
        bp = window_size is not None
        cfg = self._cfg(p, window_mode=L.WINDOW_BP if bp else L.WINDOW_SNPS,
                        window=int(window_size if bp else snp_window_size), bg_mode=L.BG_PER_CHROM, fst=True)
        eng = self._engine()
        dev = eng.upload(p)
        try:
            pl = eng.plan(dev, cfg)
            try:
                pl.run()
                pl.check()
                recs, fst = pl.read(), pl.read_fst()
            finally:
                pl.close()
        finally:
            dev.close()
        return post.window_fst_labels(recs, fst, p, int(window_size if bp else snp_window_size), bp)

    # ------------------------------------------------------------------ SFS primitives
    def calculate_2d_sfs(self, data_dict):
        """2D SFS dict over the grid (140-232), accumulated on the GPU (distributed: every rank a slice
        of the SNPs, one device all-reduce -- the genome-wide background of the reference script,
        1970-1983, from sharded data)."""
        self.data_dict = data_dict
        p = self._pack(data_dict)
        n1, n2 = 2 * self.pop1_size, 2 * self.pop2_size
        if p.n == 0:
            return {(i, j): 0 for i in range(n1 + 1) for j in range(n2 + 1)}
        h2, _, _ = self._hist(p, self._cfg(p), -1)
        return {(i, j): int(h2[i, j]) for i in range(n1 + 1) for j in range(n2 + 1)}

    def calculate_1d_sfs(self, data_dict, pop, pop_size, start_position, end_position, variant_type):
        """Unfolded 1D SFS dict of raw alt counts (398-444), accumulated on the GPU."""
        self.data_dict = data_dict
        self.pop = pop
        self.pop_size = pop_size
        self.start_position = start_position
        self.end_position = end_position
        self.variant_type = variant_type
        p = self._pack(data_dict, pop1=pop, pop2=pop).single_pop(pop)
        if p.n == 0:
            return {i: 0 for i in range(2 * pop_size + 1)}
        ann = -1
        if variant_type is not None:
            ann = p.ann_names.index(variant_type) if variant_type in p.ann_names else _NO_ANN
        cfg = ScanConfig(n1p=pop_size, n2p=pop_size, fold=False, ann_want=ann,
                         start_position=None if start_position is None else int(start_position),
                         end_position=None if end_position is None else int(end_position))
        _, u1, _ = self._hist(p, cfg, -1)
        return {i: int(u1[i]) for i in range(2 * pop_size + 1)}

    def fold_1d_sfs(self, sfs_dict):
        """446-463: minor = min(f, F - f) with F = max key."""
        num_chromosomes = max(sfs_dict.keys())
        folded = {}
        for freq, count in sfs_dict.items():
            m = min(freq, num_chromosomes - freq)
            folded[m] = folded[m] + count if m in folded else count
        return folded

    @staticmethod
    def _normalize_values(values):
        total = sum(values[1:-1])
        return [v / total for v in values]

    def normalize_2d_sfs(self, sfs):
        """234-247: divide by sum(values[1:-1]) in insertion order."""
        self.sfs = sfs
        vals = self._normalize_values(list(sfs.values()))
        return dict(zip(sfs.keys(), vals))

    def normalize_1d_sfs(self, sfs):
        """465-476."""
        self.sfs = sfs
        vals = self._normalize_values(list(sfs.values()))
        return dict(zip(sfs.keys(), vals))

    def count_snps(self, window_data, variant_type):
        """291-302."""
        self.window_data = window_data
        self.variant_type = variant_type
        if variant_type is None:
            return len(window_data)
        return sum(1 for d in window_data.values() if d.get("annotation") == variant_type)

    def new_term(self, T1D, T2D):
        """779-785."""
        self.T1D = T1D
        self.T2D = T2D
        return T2D - T1D

    # dense-dict likelihoods: evaluated by the same GPU kernel on a synthetic SNP stream that
    # reproduces the given foreground spectrum (one SNP per count, no fold)
    def calculate_likelihood_2D(self, foreground_2d_sfs, background_2d_sfs):
        """625-684."""
        self.foreground_2d_sfs = foreground_2d_sfs
        self.background_2d_sfs = background_2d_sfs
        from sfs2d.dense import clr_2d
        return clr_2d(self._engine(), foreground_2d_sfs, background_2d_sfs, guards=True)

    def calculate_likelihood_1D(self, foreground_sfs, background_sfs):
        """478-537."""
        self.foreground_sfs = foreground_sfs
        self.background_sfs = background_sfs
        from sfs2d.dense import clr_1d
        return clr_1d(self._engine(), foreground_sfs, background_sfs, guards=True)

    # ------------------------------------------------------------------ helpers
    def _bg2d_array(self, bg):
        n1, n2 = 2 * self.pop1_size, 2 * self.pop2_size
        out = np.zeros((n1 + 1) * (n2 + 1), np.float64)
        keys = [(i, j) for i in range(n1 + 1) for j in range(n2 + 1)]
        for k, key in enumerate(keys[1:-1], start=1):
            out[k] = bg[key]            # background_2d_sfs[k] for k in bins[1:-1] (:658-661)
        return out

    @staticmethod
    def _bg1d_array(bg, pop_size):
        out = np.zeros(pop_size + 1, np.float64)
        for k in range(1, pop_size):
            out[k] = bg[k]              # background_sfs[k] for k in bins[1:-1] (:505-508)
        return out
