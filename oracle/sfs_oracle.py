"""CPU oracle: a plain numpy/scipy restatement of the reference's window scan.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker.  The product path (``2dsfs-scan_amd/``) never imports it.

Parity pin: every driver below is checked against golden vectors produced by the
reference's own, unmodified functions (``tests/golden/gen_golden.py``, run in the
build container where ``/root/reference`` is mounted) and against the reference's
published CSVs (``data/ECBstats_*.csv`` chr1 rows).  See ``tests/test_oracle_golden.py``.

It restates, on the packed SoA arrays of ``sfs2d.pack.PackedSNPs``, the dense
per-window algorithm of ``scripts/src/twoDSFS_class.py`` (class
``LikelihoodInference_jointSFS``) and ``scripts/sims_scan.py``:

* 2D SFS with joint fold ........ twoDSFS_class.py:140-232  (sims_scan.py:123-234)
* 1D SFS / fold ................. twoDSFS_class.py:398-463  (sims_scan.py:262-322)
* normalisation ................. twoDSFS_class.py:234-247, 465-476
* multinomial CLR T1D / T2D ..... twoDSFS_class.py:478-537, 625-684 (sims_scan.py:325-440)
* drivers (windows, bg, quirks) . T1D_scan 539-623, T2D_scan 686-776,
                                  combined_scan 787-991, scan_chooseChr 993-1159,
                                  scan_precomputed_BG 1161-1299,
                                  scan_chooseChr_bySNPs 1303-1420,
                                  scan_perChr_bySNPs 1422-1541,
                                  sims_scan.process_window 451-590

The arithmetic lives in scipy.stats.multinomial.logpmf (scipy 1.15.3 here), which
the reference calls; the oracle calls the same function on the same dense vectors.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
from scipy.stats import multinomial


class Cfg:
    """The constructor state the reference methods read (twoDSFS_class.py:21-33)."""

    def __init__(self, pop1_size=18, pop2_size=14, variant_type=None, fold=True,
                 start_position=None, end_position=None):
        self.n1p = int(pop1_size)
        self.n2p = int(pop2_size)
        self.variant_type = variant_type
        self.fold = bool(fold)
        self.start_position = None if start_position is None else int(start_position)
        self.end_position = None if end_position is None else int(end_position)


# ----------------------------------------------------------------------------- SFS

def _sfs_mask(p, idx, cfg, use_pos_filter=True):
    m = np.ones(len(idx), dtype=bool)
    if use_pos_filter:
        pos = p.pos[idx].astype(np.int64)
        if cfg.start_position is not None:
            m &= pos >= cfg.start_position          # twoDSFS_class.py:179-180
        if cfg.end_position is not None:
            m &= pos <= cfg.end_position            # :181-182
    vm = p.variant_mask(cfg.variant_type)           # :185-187
    if vm is not None:
        m &= vm[idx].astype(bool)
    return m


def sfs2d(p, idx, cfg) -> np.ndarray:
    """Dense (2*n1p+1, 2*n2p+1) int64 grid; twoDSFS_class.py:140-232."""
    n1, n2 = 2 * cfg.n1p, 2 * cfg.n2p
    idx = np.asarray(idx, dtype=np.int64)
    m = _sfs_mask(p, idx, cfg)
    r1, a1, r2, a2 = p.ref1[idx], p.alt1[idx], p.ref2[idx], p.alt2[idx]
    if cfg.fold:                                     # :197-206 joint fold on individual counts
        sw = (a1 + a2) > (cfg.n1p + cfg.n2p)
        a1 = np.where(sw, r1, a1)
        a2 = np.where(sw, r2, a2)
    keep = m & ~((a1 == 0) & (a2 == 0))              # :212-213
    a1k, a2k = a1[keep], a2[keep]
    if a1k.size and (a1k.max() > n1 or a2k.max() > n2):
        raise ValueError("2D SFS bin outside the (2*pop1_size+1)x(2*pop2_size+1) grid "
                         "(allele counts exceed the declared sample size)")
    flat = np.bincount(a1k * (n2 + 1) + a2k, minlength=(n1 + 1) * (n2 + 1))
    return flat.reshape(n1 + 1, n2 + 1).astype(np.int64)


def sfs1d(p, idx, which, cfg, use_pos_filter=True) -> np.ndarray:
    """Unfolded 1D SFS int64[2*pop_size+1] of raw alt counts; twoDSFS_class.py:398-444."""
    npop = cfg.n1p if which == 1 else cfg.n2p
    idx = np.asarray(idx, dtype=np.int64)
    m = _sfs_mask(p, idx, cfg, use_pos_filter)
    alt = (p.alt1 if which == 1 else p.alt2)[idx]
    keep = m & (alt != 0)                             # :430-431
    ak = alt[keep]
    if ak.size and ak.max() > 2 * npop:
        raise KeyError(int(ak.max()))                 # sfs_dict[alt_count] += 1 on a missing key
    return np.bincount(ak, minlength=2 * npop + 1).astype(np.int64)


def fold1d(sfs: np.ndarray) -> np.ndarray:
    """twoDSFS_class.py:446-463: minor = min(f, F - f), F = max key = 2*pop_size."""
    F = len(sfs) - 1
    out = np.zeros(F // 2 + 1, dtype=sfs.dtype)
    for f, c in enumerate(sfs):
        out[min(f, F - f)] += c
    return out


def normalize(values_in_insertion_order: np.ndarray) -> np.ndarray:
    """normalize_2d_sfs / normalize_1d_sfs (234-247, 465-476): divide by sum(values[1:-1])."""
    vals = [int(v) if isinstance(v, (np.integer,)) else v for v in values_in_insertion_order.tolist()]
    total = sum(vals[1:-1])
    return np.array([v / total for v in vals], dtype=np.float64)


# ----------------------------------------------------------------------------- CLR

def clr(x_inner, bg_inner, guards=True):
    """calculate_likelihood_2D / _1D with the reference's exact list arithmetic.

    x_inner: int counts of the window at bins[1:-1]; bg_inner: background values at the same
    bins (ints or floats).  guards=True: return None on empty fg / bg (twoDSFS_class.py:497-499,
    520-522, 645-647, 668-670); guards=False: the sims variant (sims_scan.py:325-440), which
    raises ZeroDivisionError instead."""
    counts_fg = [int(c) for c in x_inner]
    total_fg = sum(counts_fg)
    if guards and total_fg == 0:
        return None
    p_fg = [c / total_fg for c in counts_fg]
    counts_bg = [(int(b) if isinstance(b, (int, np.integer)) else float(b)) for b in bg_inner]
    total_bg = sum(counts_bg)
    if guards and total_bg == 0:
        return None
    p_bg = [c / total_bg for c in counts_bg]
    ll_bg = multinomial.logpmf(x=counts_fg, n=total_fg, p=p_bg)
    ll_fg = multinomial.logpmf(x=counts_fg, n=total_fg, p=p_fg)
    return 2 * (ll_fg - ll_bg)


def clr2d(fg_grid, bg_grid, guards=True):
    """bins = sorted(keys) of the full grid -> row-major flat order; bins[1:-1] (:630-635)."""
    return clr(fg_grid.ravel()[1:-1], np.asarray(bg_grid).ravel()[1:-1], guards)


def clr1d(fg_folded, bg_1d, guards=True):
    """fg folded keys 0..pop_size sorted; bins[1:-1] = 1..pop_size-1 (:486-488); bg[k] read
    by key, so an unfolded bg (sims quirk Q7) is read at raw counts 1..pop_size-1."""
    k = len(fg_folded) - 1
    return clr(fg_folded[1:k], np.asarray(bg_1d)[1:k], guards)


def _num(v):
    return None if v is None else float(v)


# ----------------------------------------------------------------------------- windows

def bp_windows(p, ws):
    """Fixed-bp segmentation exactly as the reference loop (twoDSFS_class.py:843-949).

    Returns [(chrom_idx, window_start, snp_begin, snp_end)] in scan order."""
    out = []
    for c in range(p.nchrom):
        s, e = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
        if s == e:
            continue
        pos = p.pos[s:e].astype(np.int64)
        start = 1
        b = s
        for i in range(s, e):
            q = int(pos[i - s])
            if q < start + ws:
                continue
            if i > b:
                out.append((c, start, b, i))
            start += ws * ((q - start) // ws)
            b = i
        out.append((c, start, b, e))
    return out


def snp_windows(p, S):
    """Fixed-SNP-count windows (twoDSFS_class.py:1515-1535): every S SNPs per chromosome;
    label start = first pos, then previous end + 1; end = last SNP's pos; tail dropped."""
    out, skipped = [], []
    for c in range(p.nchrom):
        s, e = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
        start_pos = int(p.pos[s]) if e > s else None
        i = s
        while i + S <= e:
            endp = int(p.pos[i + S - 1])
            out.append((c, start_pos, endp, i, i + S))
            start_pos = endp + 1
            i += S
        if i < e:
            skipped.append((c, start_pos, i, e))
    return out, skipped


def count_snps(p, b, e, cfg):
    vm = p.variant_mask(cfg.variant_type)
    return (e - b) if vm is None else int(vm[b:e].sum())


# ----------------------------------------------------------------------------- drivers

def chrom_backgrounds(p, cfg):
    bg = []
    for c in range(p.nchrom):
        idx = np.arange(p.chrom_off[c], p.chrom_off[c + 1])
        bg.append((sfs2d(p, idx, cfg), fold1d(sfs1d(p, idx, 1, cfg)), fold1d(sfs1d(p, idx, 2, cfg))))
    return bg


def _stats(p, b, e, cfg, bgs, guards=True):
    idx = np.arange(b, e)
    T2D = clr2d(sfs2d(p, idx, cfg), bgs[0], guards)
    f1 = fold1d(sfs1d(p, idx, 1, cfg))
    f2 = fold1d(sfs1d(p, idx, 2, cfg))
    return T2D, f1, f2


def combined_scan(p, ws, cfg) -> Dict[str, dict]:
    """twoDSFS_class.py:787-991 with quirks Q5 (per-chrom bg), Q6 (stale carry), Q9 (last window)."""
    bgs = chrom_backgrounds(p, cfg)
    wins = bp_windows(p, ws)
    res: Dict[str, dict] = {}
    st = {}

    def get(name):
        if name not in st:
            raise UnboundLocalError(f"local variable '{name}' referenced before assignment")
        return st[name]

    for w, (c, start, b, e) in enumerate(wins):
        label = f"{p.chrom_names[c]} {start}-{start + ws - 1}"
        if w < len(wins) - 1:
            T2D, f1, f2 = _stats(p, b, e, cfg, bgs[c])
            st["T2D"] = T2D
            st["folded_fg_sfs_pop1"] = f1
            st["T1D_pop1"] = clr1d(f1, bgs[c][1])
            st["folded_fg_sfs_pop2"] = f2
            st["T1D_pop2"] = clr1d(f2, bgs[c][2])
            if st["T2D"] and st["T1D_pop1"] and st["T1D_pop2"] is not None:
                st["new_term_pop1"] = st["T2D"] - st["T1D_pop1"]
                st["new_term_pop2"] = st["T2D"] - st["T1D_pop2"]
                st["T2D_diff"] = st["T2D"] - (st["T1D_pop1"] + st["T1D_pop2"]) / 2
            res[label] = {"snp_count": count_snps(p, b, e, cfg), "T2D": get("T2D"),
                          "T1D_pop1": get("T1D_pop1"), "T1D_pop2": get("T1D_pop2"),
                          "new_term_pop1": get("new_term_pop1"), "new_term_pop2": get("new_term_pop2"),
                          "T2D_diff": get("T2D_diff")}
        else:  # mis-indented final block, twoDSFS_class.py:951-989
            idx = np.arange(b, e)
            st["T2D"] = clr2d(sfs2d(p, idx, cfg), bgs[c][0])
            if get("T2D") is not None:
                st["folded_fg_sfs_pop1"] = fold1d(sfs1d(p, idx, 1, cfg))
            if get("T1D_pop1") is not None:
                st["T1D_pop1"] = clr1d(get("folded_fg_sfs_pop1"), bgs[c][1])
                st["folded_fg_sfs_pop2"] = fold1d(sfs1d(p, idx, 2, cfg))
            if get("T1D_pop2") is not None:
                st["T1D_pop2"] = clr1d(get("folded_fg_sfs_pop2"), bgs[c][2])
                if st["T2D"] and st["T1D_pop1"] and st["T1D_pop2"] is not None:
                    st["new_term_pop1"] = st["T2D"] - st["T1D_pop1"]
                    st["new_term_pop2"] = st["T2D"] - st["T1D_pop2"]
                    st["T2D_diff"] = st["T2D"] - (st["T1D_pop1"] + st["T1D_pop2"]) / 2
                res[label] = {"snp_count": count_snps(p, b, e, cfg), "T2D": get("T2D"),
                              "T1D_pop1": get("T1D_pop1"), "T1D_pop2": get("T1D_pop2"),
                              "new_term_pop1": get("new_term_pop1"), "new_term_pop2": get("new_term_pop2"),
                              "T2D_diff": get("T2D_diff")}
    if not wins:
        get("T2D")  # empty input: `if T2D is not None` on an unbound local
    return res


def _fixed_bg_scan(p, ws, cfg, bg2, bg1a, bg1b):
    """Shared body of scan_chooseChr (993-1159) and scan_precomputed_BG (1161-1299)."""
    res = {}
    for (c, start, b, e) in bp_windows(p, ws):
        idx = np.arange(b, e)
        T2D = clr2d(sfs2d(p, idx, cfg), bg2)
        T1 = clr1d(fold1d(sfs1d(p, idx, 1, cfg)), bg1a)
        T2 = clr1d(fold1d(sfs1d(p, idx, 2, cfg)), bg1b)
        nt1 = T2D - T1   # TypeError when a statistic is None, as in the reference (1071-1072)
        nt2 = T2D - T2
        res[f"{p.chrom_names[c]} {start}-{start + ws - 1}"] = {
            "snp_count": count_snps(p, b, e, cfg), "T2D": T2D, "T1D_pop1": T1, "T1D_pop2": T2,
            "new_term_pop1": nt1, "new_term_pop2": nt2}
    return res


def scan_chooseChr(p, ws, bg_chrom, cfg):
    if bg_chrom not in p.chrom_names:
        raise ValueError(f"Background chromosome {bg_chrom} not found in the data.")
    c = p.chrom_names.index(bg_chrom)
    idx = np.arange(p.chrom_off[c], p.chrom_off[c + 1])
    return _fixed_bg_scan(p, ws, cfg, sfs2d(p, idx, cfg), fold1d(sfs1d(p, idx, 1, cfg)),
                          fold1d(sfs1d(p, idx, 2, cfg)))


def scan_precomputed_BG(p, ws, bg2, bg1a, bg1b, cfg):
    return _fixed_bg_scan(p, ws, cfg, np.asarray(bg2), np.asarray(bg1a), np.asarray(bg1b))


def genome_backgrounds_normalized(p, cfg):
    """Script cell twoDSFS_class.py:1970-1981: whole-data 2D / folded 1D, normalised."""
    idx = np.arange(p.n)
    g2 = normalize(sfs2d(p, idx, cfg).ravel()).reshape(2 * cfg.n1p + 1, 2 * cfg.n2p + 1)
    g1a = normalize(fold1d(sfs1d(p, idx, 1, cfg)))
    g1b = normalize(fold1d(sfs1d(p, idx, 2, cfg)))
    return g2, g1a, g1b


def _bysnp_scan(p, S, cfg, bg_for_chrom, with_diff):
    res = {}
    wins, _ = snp_windows(p, S)
    for (c, start, endp, b, e) in wins:
        idx = np.arange(b, e)
        fg2 = sfs2d(p, idx, cfg)
        if fg2.sum() == 0:                           # :1376 / :1496
            continue
        bg2, bg1a, bg1b = bg_for_chrom(c)
        T2D = clr2d(fg2, bg2)
        T1 = clr1d(fold1d(sfs1d(p, idx, 1, cfg)), bg1a)
        T2 = clr1d(fold1d(sfs1d(p, idx, 2, cfg)), bg1b)
        rec = {"snp_count": S, "T2D": T2D, "T1D_pop1": T1, "T1D_pop2": T2,
               "new_term_pop1": T2D - T1, "new_term_pop2": T2D - T2}
        if with_diff:
            rec["T2D_diff"] = T2D - (T1 + T2) / 2
        res[f"{p.chrom_names[c]} {start}-{endp}"] = rec
    return res


def scan_chooseChr_bySNPs(p, S, bg_chrom, cfg):
    if bg_chrom not in p.chrom_names:
        raise ValueError(f"Background chromosome {bg_chrom} not found in the data.")
    c = p.chrom_names.index(bg_chrom)
    idx = np.arange(p.chrom_off[c], p.chrom_off[c + 1])
    bg2 = normalize(sfs2d(p, idx, cfg).ravel())
    bg1a = normalize(fold1d(sfs1d(p, idx, 1, cfg)))
    bg1b = normalize(fold1d(sfs1d(p, idx, 2, cfg)))
    return _bysnp_scan(p, S, cfg, lambda _c: (bg2, bg1a, bg1b), with_diff=False)


def scan_perChr_bySNPs(p, S, cfg):
    bgs = chrom_backgrounds(p, cfg)
    return _bysnp_scan(p, S, cfg, lambda c: bgs[c], with_diff=True)


def T1D_scan(p, ws, bg1d, pop, pop_size, cfg):
    """twoDSFS_class.py:539-623: fixed-bp windows, calculate_1d_sfs of ``pop`` (raw alt counts, the
    constructor's filters), fold_1d_sfs, calculate_likelihood_1D against the supplied ``bg1d``."""
    which = 1 if pop == p.pop1 else (2 if pop == p.pop2 else 0)
    c1 = Cfg(pop_size, pop_size, cfg.variant_type, cfg.fold, cfg.start_position, cfg.end_position)
    res = {}
    for (c, start, b, e) in bp_windows(p, ws):
        idx = np.arange(b, e)
        if which:
            u = sfs1d(p, idx, which, c1)
        else:   # calls.get(pop, (0, 0)): no SNP enters the spectrum
            u = np.zeros(2 * pop_size + 1, np.int64)
        res[f"{p.chrom_names[c]} {start}-{start + ws - 1}"] = {
            "snp_count": count_snps(p, b, e, cfg), "T1D": clr1d(fold1d(u), bg1d)}
    return res


def T2D_scan(p, ws, bg2, cfg, last=None):
    """twoDSFS_class.py:686-776, restated as the reference's own loop over the sorted SNPs with a
    window dict keyed by SNP.  At each chromosome change the per-chromosome background loop (:740)
    rebinds ``snp_key`` to the data dict's last key (``last``: its index in p; default the last SNP,
    the order to_snp_dict inserts), so that key -- its calls, annotation and key position -- enters
    the window in place of the chromosome's first SNP (:748 / :763).  Scored against the supplied
    ``bg2`` (:753, :768)."""
    last = p.n - 1 if last is None else int(last)
    chrom = p.chrom_of()
    res = {}
    cur, start, win = None, 0, {}

    def emit():
        idx = np.array(list(win), dtype=np.int64)   # keys = SNP indices; sfs2d filters by p.pos[key]
        res[f"{p.chrom_names[cur]} {start}-{start + ws - 1}"] = {
            "snp_count": count_snps_idx(p, idx, cfg), "T2D": clr2d(sfs2d(p, idx, cfg), bg2)}

    for i in range(p.n):
        c, q, key = int(chrom[i]), int(p.pos[i]), i
        if c != cur:
            if win:
                emit()
            cur, start, win = c, 1, {}
            key = last
        if q < start + ws:
            win[key] = True
        else:
            if win:
                emit()
            start += ws * ((q - start) // ws)
            win = {key: True}
    if win:
        emit()
    return res


def count_snps_idx(p, idx, cfg):
    vm = p.variant_mask(cfg.variant_type)
    return len(idx) if vm is None else int(vm[idx].sum())


def sims_backgrounds(p, n1p, n2p, start=0, end=500000, variant_type=None):
    """sims_scan.py:615-617: 2D folded bg and UNFOLDED 1D bgs over pos in [start, end]."""
    cfg = Cfg(n1p, n2p, variant_type, True, start, end)
    idx = np.arange(p.n)
    return sfs2d(p, idx, cfg), sfs1d(p, idx, 1, cfg), sfs1d(p, idx, 2, cfg)


def sims_process_window(p, bg2, bg1, bg2b, ws, n1p, n2p, start=None, end=None, variant_type=None):
    """sims_scan.py:451-590: no None guards (ZeroDivisionError), T2D_diff with MINUS (Q7)."""
    cfg = Cfg(n1p, n2p, variant_type, True, start, end)
    res = {}
    for (c, ws0, b, e) in bp_windows(p, ws):
        idx = np.arange(b, e)
        T2D = clr2d(sfs2d(p, idx, cfg), bg2, guards=False)
        T1 = clr1d(fold1d(sfs1d(p, idx, 1, cfg)), bg1, guards=False)
        T2 = clr1d(fold1d(sfs1d(p, idx, 2, cfg)), bg2b, guards=False)
        res[f"{p.chrom_names[c]} {ws0}-{ws0 + ws - 1}"] = {
            "window_type": "background" if 0 <= ws0 < 500000 else "foreground",
            "window_start": ws0, "window_end": ws0 + ws,
            "snp_count": count_snps(p, b, e, cfg), "T2D": T2D, "T1D_p1": T1, "T1D_p2": T2,
            "new_term_p1": T2D - T1, "new_term_p2": T2D - T2, "T2D_diff": T2D - (T1 - T2) / 2}
    return res


# ----------------------------------------------------------------------------- records

def window_records(p, wins, cfg, bg_of_window, guards=True):
    """Per-window raw statistics (the quantities the HIP scan emits before the host post-pass):
    snp_count, N2, N1a, N1b, T2D, T1D_p1, T1D_p2 for each (c, start, b, e) window."""
    out = []
    for w in wins:
        c, b, e = w[0], w[-2], w[-1]
        idx = np.arange(b, e)
        bg2, bg1a, bg1b = bg_of_window(c)
        g = sfs2d(p, idx, cfg)
        f1 = fold1d(sfs1d(p, idx, 1, cfg))
        f2 = fold1d(sfs1d(p, idx, 2, cfg))
        out.append(dict(snp_count=count_snps(p, b, e, cfg), N2=int(g.ravel()[1:-1].sum()),
                        N2_all=int(g.sum()), N1a=int(f1[1:-1].sum()), N1b=int(f2[1:-1].sum()),
                        T2D=_num(clr2d(g, bg2, guards)), T1D_p1=_num(clr1d(f1, bg1a, guards)),
                        T1D_p2=_num(clr1d(f2, bg1b, guards))))
    return out


def window_fst(p, idx, cfg) -> Optional[float]:
    """Hudson's Fst (Bhatia et al. 2013, ratio of averages) of one window -- NOT part of the
    reference (its published Fst is pixy's Weir-Cockerham, joined in R): parity is
    unpinned, this restatement defines it.  SNPs: those entering the window's 2D SFS (filters
    passed, (0,0) after the joint fold excluded; twoDSFS_class.py:179-217) with >= 2 called alleles
    in each population; raw (unfolded) frequencies p = alt / (ref + alt):
        num = (p1 - p2)^2 - p1(1-p1)/(n1c-1) - p2(1-p2)/(n2c-1),  den = p1(1-p2) + p2(1-p1),
    Fst = sum(num) / sum(den); None when no SNP qualifies or sum(den) == 0."""
    idx = np.asarray(idx, dtype=np.int64)
    m = _sfs_mask(p, idx, cfg)
    r1, a1, r2, a2 = p.ref1[idx], p.alt1[idx], p.ref2[idx], p.alt2[idx]
    x1, x2 = a1, a2
    if cfg.fold:
        sw = (a1 + a2) > (cfg.n1p + cfg.n2p)
        x1 = np.where(sw, r1, a1)
        x2 = np.where(sw, r2, a2)
    n1c, n2c = r1 + a1, r2 + a2
    keep = m & ~((x1 == 0) & (x2 == 0)) & (n1c >= 2) & (n2c >= 2)
    if not keep.any():
        return None
    n1c, n2c = n1c[keep].astype(np.float64), n2c[keep].astype(np.float64)
    p1 = a1[keep] / n1c
    p2 = a2[keep] / n2c
    num = (p1 - p2) ** 2 - p1 * (1 - p1) / (n1c - 1) - p2 * (1 - p2) / (n2c - 1)
    den = p1 * (1 - p2) + p2 * (1 - p1)
    d = float(den.sum())
    return None if d == 0.0 else float(num.sum()) / d
