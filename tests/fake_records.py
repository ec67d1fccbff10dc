"""Test-only: build the records a plan would emit, from the CPU oracle, so the host post-pass
(sfs2d.post) can be checked on a machine without a GPU."""
import numpy as np

from oracle import sfs_oracle as O
from sfs2d import _lib as L


def _fill(rec, o, flags=0):
    rec["snp_count"], rec["n2"], rec["n2_all"], rec["n1a"], rec["n1b"] = (
        o["snp_count"], o["N2"], o["N2_all"], o["N1a"], o["N1b"])
    rec["t2d"] = 0.0 if o["T2D"] is None else o["T2D"]
    rec["t1d_p1"] = 0.0 if o["T1D_p1"] is None else o["T1D_p1"]
    rec["t1d_p2"] = 0.0 if o["T1D_p2"] is None else o["T1D_p2"]
    rec["flags"] = flags


def _bgflags(bg2, bg1a, bg1b, n1p, n2p):
    f = 0
    if np.asarray(bg2).ravel()[1:-1].sum() == 0:
        f |= L.W_BG2_ZERO
    if np.asarray(bg1a)[1:n1p].sum() == 0:
        f |= L.W_BG1A_ZERO
    if np.asarray(bg1b)[1:n2p].sum() == 0:
        f |= L.W_BG1B_ZERO
    return f


def bp_records(p, ws, ocfg, bg_of_chrom, prev_extra=False):
    """Dense fixed-bp slots (empty ones flagged), + the Q9 helper record."""
    wins = O.bp_windows(p, ws)
    slot_base = [0]
    for c in range(p.nchrom):
        s, e = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
        ns = 0 if s == e else ((int(p.pos[e - 1]) - 1) // ws if p.pos[e - 1] else 0) + 1
        slot_base.append(slot_base[-1] + ns)
    nslots = slot_base[-1]
    recs = np.zeros(nslots + (1 if prev_extra and wins else 0), dtype=L.WINDOW_DTYPE)
    recs["flags"] = L.W_EMPTY
    for c in range(p.nchrom):
        for s in range(slot_base[c], slot_base[c + 1]):
            recs[s]["chrom"] = c
            recs[s]["wid"] = s - slot_base[c]
    ref = O.window_records(p, wins, ocfg, bg_of_chrom)
    for (c, start, b, e), o in zip(wins, ref):
        s = slot_base[c] + (start - 1) // ws
        r = recs[s]
        r["chrom"], r["begin"], r["end"] = c, b, e
        bg = bg_of_chrom(c)
        _fill(r, o, _bgflags(*bg, ocfg.n1p, ocfg.n2p))
        recs[s] = r
    if prev_extra and wins:
        r = recs[nslots]
        r["flags"] = L.W_EXTRA
        if len(wins) >= 2:
            c_last = wins[-1][0]
            cp, _, b, e = wins[-2]
            o = O.window_records(p, [wins[-2]], ocfg, lambda _c: bg_of_chrom(c_last))[0]
            r["chrom"], r["begin"], r["end"] = cp, b, e
            _fill(r, o, L.W_EXTRA | _bgflags(*bg_of_chrom(c_last), ocfg.n1p, ocfg.n2p))
        else:
            r["flags"] = L.W_EXTRA | L.W_EMPTY
        recs[nslots] = r
    return recs


def snp_records(p, S, ocfg, bg_of_chrom):
    wins, _ = O.snp_windows(p, S)
    recs = np.zeros(len(wins), dtype=L.WINDOW_DTYPE)
    ref = O.window_records(p, [(w[0], w[3], w[4]) for w in wins], ocfg, bg_of_chrom)
    for k, ((c, sp, ep, b, e), o) in enumerate(zip(wins, ref)):
        r = recs[k]
        r["chrom"], r["begin"], r["end"] = c, b, e
        r["wid"] = (b - int(p.chrom_off[c])) // S          # the window's index in its chromosome
        _fill(r, o, _bgflags(*bg_of_chrom(c), ocfg.n1p, ocfg.n2p))
        recs[k] = r
    return recs
