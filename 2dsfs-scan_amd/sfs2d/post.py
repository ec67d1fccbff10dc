"""Host post-pass: window records -> the reference's result dicts.

The HIP scan emits one record per window (statistics against the window's background plus
the counts that decide the reference's None / error cases).  What remains is sequential,
O(windows) bookkeeping that the reference performs in its Python driver loops and that must be
reproduced exactly:

* None rules: N == 0 or background inner sum == 0 -> None (twoDSFS_class.py:497-499, 520-522,
  645-647, 668-670); the sims functions raise ZeroDivisionError instead (sims_scan.py:325-440).
* combined_scan's stale carry (quirk Q6, :875 / :930): derived terms are only refreshed when
  ``T2D and T1D_pop1 and T1D_pop2 is not None`` -- truthiness, so an exact 0.0 keeps the previous
  window's new_term / T2D_diff, and a failing first window raises UnboundLocalError.
* combined_scan's mis-indented final block (quirk Q9, :951-989).
* scan_chooseChr / scan_precomputed_BG: ``T2D - T1D`` with no guard (TypeError on None, :1071).
* scan_*_bySNPs: windows of exactly S SNPs, labels, skip-if-empty, warnings (:1303-1541).
* sims_scan.process_window: window_type / window_start / window_end and MINUS in T2D_diff (Q7).
Every arithmetic on the statistics here is the reference's own Python float expression.
"""
from __future__ import annotations

import numpy as np

from . import _lib as L


def _v(r, which):
    """Statistic of a record as the reference would hold it (None or float)."""
    if which == 2:
        return None if (r["n2"] == 0 or r["flags"] & L.W_BG2_ZERO) else float(r["t2d"])
    if which == 1:
        return None if (r["n1a"] == 0 or r["flags"] & L.W_BG1A_ZERO) else float(r["t1d_p1"])
    return None if (r["n1b"] == 0 or r["flags"] & L.W_BG1B_ZERO) else float(r["t1d_p2"])


def num_slots(recs):
    """Records of a plan are its window slots, plus one trailing Q9 helper when requested."""
    return len(recs) - 1 if len(recs) and (recs[-1]["flags"] & L.W_EXTRA) else len(recs)


def _windows(recs, nslots):
    body = recs[:nslots]
    return body[(body["flags"] & L.W_EMPTY) == 0]


class _Locals:
    """The driver's local variables; reading an unassigned one raises like CPython."""

    def __init__(self):
        self.d = {}

    def __getitem__(self, k):
        try:
            return self.d[k]
        except KeyError:
            raise UnboundLocalError(f"local variable '{k}' referenced before assignment") from None

    def __setitem__(self, k, v):
        self.d[k] = v


def combined_scan(recs, packed, ws, nslots):
    """twoDSFS_class.py:787-991 (per-chromosome background)."""
    wins = _windows(recs, nslots)
    extra = recs[nslots] if len(recs) > nslots else None
    names = packed.chrom_names
    res = {}
    st = _Locals()
    nw = len(wins)

    def label(r):
        s = 1 + int(r["wid"]) * ws
        return f"{names[int(r['chrom'])]} {s}-{s + ws - 1}"

    def derive():
        if st["T2D"] and st["T1D_pop1"] and st["T1D_pop2"] is not None:
            st["new_term_pop1"] = st["T2D"] - st["T1D_pop1"]
            st["new_term_pop2"] = st["T2D"] - st["T1D_pop2"]
            st["T2D_diff"] = st["T2D"] - (st["T1D_pop1"] + st["T1D_pop2"]) / 2

    def record(r):
        return {"snp_count": int(r["snp_count"]), "T2D": st["T2D"], "T1D_pop1": st["T1D_pop1"],
                "T1D_pop2": st["T1D_pop2"], "new_term_pop1": st["new_term_pop1"],
                "new_term_pop2": st["new_term_pop2"], "T2D_diff": st["T2D_diff"]}

    for w in range(nw - 1):
        r = wins[w]
        st["T2D"] = _v(r, 2)
        st["T1D_pop1"] = _v(r, 1)
        st["T1D_pop2"] = _v(r, 0)
        derive()
        res[label(r)] = record(r)
    if nw == 0:
        st["T2D"]   # `if T2D is not None` on an unbound local (empty input)
        return res
    # final block (:951-989): T2D of the last window; T1D_pop1 / T1D_pop2 are recomputed only
    # behind the PREVIOUS window's values, from whichever folded spectra are bound at that point
    f = wins[nw - 1]
    st["T2D"] = _v(f, 2)
    pop1_from_last = st["T2D"] is not None
    if st["T1D_pop1"] is not None:
        if pop1_from_last:
            st["T1D_pop1"] = _v(f, 1)
        else:  # previous window's folded pop1 spectrum against the last chromosome's background
            st["T1D_pop1"] = _v(extra, 1)
        pop2_from_last = True
    else:
        pop2_from_last = False
    if st["T1D_pop2"] is not None:
        st["T1D_pop2"] = _v(f, 0) if pop2_from_last else _v(extra, 0)
        derive()
        res[label(f)] = record(f)
    return res


def fixed_bg_scan(recs, packed, ws, nslots):
    """scan_chooseChr (993-1159) / scan_precomputed_BG (1161-1299): one background, no guard."""
    names = packed.chrom_names
    res = {}
    for r in _windows(recs, nslots):
        T2D, T1, T2 = _v(r, 2), _v(r, 1), _v(r, 0)
        nt1 = T2D - T1
        nt2 = T2D - T2
        s = 1 + int(r["wid"]) * ws
        res[f"{names[int(r['chrom'])]} {s}-{s + ws - 1}"] = {
            "snp_count": int(r["snp_count"]), "T2D": T2D, "T1D_pop1": T1, "T1D_pop2": T2,
            "new_term_pop1": nt1, "new_term_pop2": nt2}
    return res


def single_stat_scan(recs, packed, ws, nslots, which, name):
    """T1D_scan (539-623) / T2D_scan (686-776): {label: {"snp_count", name}} per non-empty fixed-bp
    window, the statistic None for an empty window or background (no guard, no derived terms).
    which: 2 = T2D, 1 = the first population's T1D."""
    names = packed.chrom_names
    res = {}
    for r in _windows(recs, nslots):
        s = 1 + int(r["wid"]) * ws
        res[f"{names[int(r['chrom'])]} {s}-{s + ws - 1}"] = {"snp_count": int(r["snp_count"]), name: _v(r, which)}
    return res


def bysnp_scan(recs, packed, S, with_diff, final_warning):
    """scan_chooseChr_bySNPs (1303-1420) / scan_perChr_bySNPs (1422-1541)."""
    names = packed.chrom_names
    pos = packed.pos
    off = packed.chrom_off
    res = {}
    by_chrom = {}
    for r in recs:
        by_chrom.setdefault(int(r["chrom"]), []).append(r)
    cur = None
    last_start = None
    last_pos = None
    leftover = 0
    for c in range(packed.nchrom):
        s, e = int(off[c]), int(off[c + 1])
        if s == e:
            continue
        if cur is not None and leftover:
            # process_window() on the incomplete tail at a chromosome change: prints, skips
            print(f"Warning: Skipping incomplete window {names[cur]} {last_start}-{int(pos[s])} "
                  f"with {leftover} SNPs (expected {S}).")
        start = int(pos[s])
        for r in by_chrom.get(c, []):
            b, en = int(r["begin"]), int(r["end"])
            endp = int(pos[en - 1])
            if r["n2_all"] != 0:
                T2D, T1, T2 = _v(r, 2), _v(r, 1), _v(r, 0)
                rec = {"snp_count": S, "T2D": T2D, "T1D_pop1": T1, "T1D_pop2": T2,
                       "new_term_pop1": T2D - T1, "new_term_pop2": T2D - T2}
                if with_diff:
                    rec["T2D_diff"] = T2D - (T1 + T2) / 2
                res[f"{names[c]} {start}-{endp}"] = rec
            start = endp + 1
        cur = c
        last_start = start
        leftover = (e - s) % S
        last_pos = int(pos[e - 1])
    if final_warning and cur is not None and leftover:
        print(f"Warning: Skipping incomplete final window {names[cur]} {last_start}-{last_pos} "
              f"with {leftover} snps (expected {S}).")
    return res


def window_fst_labels(recs, fst, packed, w, bp):
    """{window label: Fst or None} in scan order; labels as combined_scan (bp windows: wid) or the
    bySNPs drivers (first SNP position - last SNP position of each complete S-SNP window) make them."""
    names = packed.chrom_names
    out = {}
    nslots = min(len(fst), num_slots(recs))
    if bp:
        for r, f in zip(recs[:nslots], fst[:nslots]):
            if r["flags"] & L.W_EMPTY:
                continue
            s = 1 + int(r["wid"]) * w
            out[f"{names[int(r['chrom'])]} {s}-{s + w - 1}"] = None if np.isnan(f) else float(f)
        return out
    pos = packed.pos
    start = {}
    for r, f in zip(recs[:nslots], fst[:nslots]):
        c = int(r["chrom"])
        st = start.get(c, int(pos[int(packed.chrom_off[c])]))
        endp = int(pos[int(r["end"]) - 1])
        if r["n2_all"] != 0:
            out[f"{names[c]} {st}-{endp}"] = None if np.isnan(f) else float(f)
        start[c] = endp + 1
    return out


def sims_process_window(recs, packed, ws, nslots):
    """sims_scan.process_window (451-590): no None guards, T2D_diff = T2D - (T1D_p1 - T1D_p2)/2."""
    names = packed.chrom_names
    res = {}
    for r in _windows(recs, nslots):
        vals = []
        for which, nfield, zflag in ((2, "n2", L.W_BG2_ZERO), (1, "n1a", L.W_BG1A_ZERO), (0, "n1b", L.W_BG1B_ZERO)):
            if r[nfield] == 0 or r["flags"] & zflag:
                raise ZeroDivisionError("division by zero")
            vals.append(_v(r, which))
        T2D, T1, T2 = vals
        s = 1 + int(r["wid"]) * ws
        res[f"{names[int(r['chrom'])]} {s}-{s + ws - 1}"] = {
            "window_type": "background" if 0 <= s < 500000 else "foreground",
            "window_start": s, "window_end": s + ws, "snp_count": int(r["snp_count"]),
            "T2D": T2D, "T1D_p1": T1, "T1D_p2": T2, "new_term_p1": T2D - T1, "new_term_p2": T2D - T2,
            "T2D_diff": T2D - (T1 - T2) / 2}
    return res
