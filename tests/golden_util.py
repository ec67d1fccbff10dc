"""Helpers to read the golden vectors (tests/golden/) and compare scan results."""
from __future__ import annotations

import json
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")

# Float contract (BASELINE.json north_star): 1e-10 relative for T1D/T2D/derived statistics.
# Differences of two statistics (new_term, T2D_diff) inherit the absolute error of their
# operands, so they are compared relative to the magnitude of the operands that formed them.
REL_TOL = 1e-10


class Golden:
    def __init__(self):
        with open(os.path.join(GOLD, "manifest.json")) as fh:
            self.manifest = json.load(fh)

    def cases(self):
        return list(self.manifest)

    def packed(self, name):
        from sfs2d.snpio import load_packed
        return load_packed(os.path.join(GOLD, f"{name}.npz"))

    def cfg(self, name):
        return self.manifest[name]["cfg"]

    def calls(self, name):
        return self.manifest[name]["calls"]

    def npz(self, fname):
        return np.load(os.path.join(GOLD, fname), allow_pickle=False)

    def published(self):
        with open(os.path.join(GOLD, "published_chr1.json")) as fh:
            return json.load(fh)


def dec(v):
    if v is None or isinstance(v, (int, bool)):
        return v
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            return v
    return v


def decode_results(enc):
    return {k: {f: dec(x) for f, x in d.items()} for k, d in enc}


def close(a, b, scale=None, rel=REL_TOL):
    """a: ours, b: reference.  Exact for None / 0.0 / inf / nan identity; else relative."""
    if b is None or a is None:
        return a is None and b is None
    if isinstance(b, str) or isinstance(a, str):
        return a == b
    a = float(a)
    b = float(b)
    if math.isnan(b) or math.isnan(a):
        return math.isnan(a) and math.isnan(b)
    if math.isinf(b) or math.isinf(a):
        return a == b
    if b == 0.0 or a == 0.0:
        return a == b  # exact zero drives the reference's truthiness guard (quirk Q6)
    s = max(abs(a), abs(b), scale or 0.0)
    return abs(a - b) <= rel * s


def compare_results(ours: dict, ref: dict, rel=REL_TOL):
    """Same keys in the same (scan) order, ints exact, floats within tolerance."""
    errs = []
    ko, kr = list(ours), list(ref)
    if ko != kr:
        missing = [k for k in kr if k not in ours][:5]
        extra = [k for k in ko if k not in ref][:5]
        errs.append(f"keys differ: {len(ko)} vs {len(kr)}; missing {missing} extra {extra}")
        return errs
    worst = 0.0
    for k in kr:
        do, dr = ours[k], ref[k]
        if list(do) != list(dr):
            errs.append(f"{k}: fields {list(do)} vs {list(dr)}")
            continue
        stat_scale = max([abs(float(dr[f])) for f in ("T2D", "T1D_pop1", "T1D_pop2", "T1D_p1", "T1D_p2")
                          if f in dr and isinstance(dr[f], float) and math.isfinite(dr[f])] + [0.0])
        for f in dr:
            vo, vr = do[f], dr[f]
            if isinstance(vr, int) and not isinstance(vr, bool) or isinstance(vr, str):
                if vo != vr:
                    errs.append(f"{k}.{f}: {vo!r} != {vr!r}")
                continue
            scale = stat_scale if f.startswith(("new_term", "T2D_diff")) else None
            if not close(vo, vr, scale, rel):
                errs.append(f"{k}.{f}: {vo!r} vs {vr!r}")
            elif isinstance(vr, float) and math.isfinite(vr) and vr != 0:
                worst = max(worst, abs(float(vo) - vr) / max(abs(vr), scale or 0.0))
    return errs if errs else []


def run_capture(fn, *a, **kw):
    import contextlib
    import io
    buf = io.StringIO()
    try:
        with contextlib.redirect_stdout(buf):
            out = fn(*a, **kw)
        return True, out, buf.getvalue()
    except Exception as e:  # noqa: BLE001
        return False, e, buf.getvalue()


def t12_inputs(p, cfgd, fn, args):
    """Inputs of a golden T2D_scan / T1D_scan call (tests/golden/gen_golden.py section F): the data
    (the packed set, or its dict with args[-1] moved to the end: T2D_scan reads the dict's last key)
    and the background dict the reference was given (whole-data 2D / folded 1D SFS with the object's
    filters, normalised for "norm"), rebuilt with the oracle.  Returns (data, bg, extra args)."""
    from oracle import sfs_oracle as O
    from sfs2d.pack import to_snp_dict
    data = p
    if args[-1] is not None:
        data = to_snp_dict(p)
        data[args[-1]] = data.pop(args[-1])
    idx = np.arange(p.n)
    if fn == "T2D_scan":
        cfg = O.Cfg(cfgd["n1p"], cfgd["n2p"], cfgd.get("variant_type"), cfgd.get("fold", True),
                    cfgd.get("start_position"), cfgd.get("end_position"))
        g = O.sfs2d(p, idx, cfg).ravel()
        vals = O.normalize(g) if args[0] == "norm" else g
        n2 = 2 * cfgd["n2p"] + 1
        bg = {(k // n2, k % n2): (float(v) if args[0] == "norm" else int(v)) for k, v in enumerate(vals)}
        return data, bg, [args[1]]
    pop, npop = args[2], args[3]
    cfg = O.Cfg(npop, npop, cfgd.get("variant_type"), cfgd.get("fold", True), cfgd.get("start_position"),
                cfgd.get("end_position"))
    which = 1 if pop == p.pop1 else (2 if pop == p.pop2 else 0)
    u = O.sfs1d(p, idx, which, cfg) if which else np.zeros(2 * npop + 1, np.int64)
    f = O.fold1d(u)
    vals = O.normalize(f) if args[0] == "norm" else f
    bg = {k: (float(v) if args[0] == "norm" else int(v)) for k, v in enumerate(vals)}
    return data, bg, [args[1], pop, npop]


def enc_value(v):
    """JSON-safe encoding of a result value (floats by repr, as tests/golden/gen_golden.py)."""
    if v is None or isinstance(v, (bool, str)):
        return v
    if isinstance(v, (int, np.integer)):
        return int(v)
    if isinstance(v, (float, np.floating)):
        return repr(float(v))
    if isinstance(v, dict):
        return {k: enc_value(x) for k, x in v.items()}
    raise TypeError(type(v))


def enc_results(res):
    return [[k, {f: enc_value(x) for f, x in d.items()}] for k, d in res.items()]
