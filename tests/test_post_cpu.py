"""Host logic on CPU: the post-pass (sfs2d.post) fed with oracle-made records reproduces the
reference drivers' outputs (golden), including quirks Q6 / Q9 and the error cases."""
import numpy as np
import pytest

import fake_records as F
import golden_util as gu
from oracle import sfs_oracle as O
from sfs2d import post


def _ocfg(cfgd):
    return O.Cfg(cfgd["n1p"], cfgd["n2p"], cfgd.get("variant_type"), cfgd.get("fold", True),
                 cfgd.get("start_position"), cfgd.get("end_position"))


def _post_call(p, cfgd, fn, args):
    ocfg = _ocfg(cfgd)
    if fn == "combined_scan":
        bgs = O.chrom_backgrounds(p, ocfg)
        recs = F.bp_records(p, args[0], ocfg, lambda c: bgs[c], prev_extra=True)
        return post.combined_scan(recs, p, args[0], post.num_slots(recs))
    if fn == "scan_perChr_bySNPs":
        bgs = O.chrom_backgrounds(p, ocfg)
        recs = F.snp_records(p, args[0], ocfg, lambda c: bgs[c])
        return post.bysnp_scan(recs, p, args[0], True, False)
    if fn == "scan_chooseChr":
        c = p.chrom_names.index(args[1])
        bg = O.chrom_backgrounds(p, ocfg)[c]
        recs = F.bp_records(p, args[0], ocfg, lambda _c: bg)
        return post.fixed_bg_scan(recs, p, args[0], post.num_slots(recs))
    if fn == "scan_precomputed_BG":
        bg = O.genome_backgrounds_normalized(p, ocfg)
        recs = F.bp_records(p, args[0], ocfg, lambda _c: bg)
        return post.fixed_bg_scan(recs, p, args[0], post.num_slots(recs))
    if fn == "scan_chooseChr_bySNPs":
        c = p.chrom_names.index(args[1])
        idx = np.arange(p.chrom_off[c], p.chrom_off[c + 1])
        bg = (O.normalize(O.sfs2d(p, idx, ocfg).ravel()), O.normalize(O.fold1d(O.sfs1d(p, idx, 1, ocfg))),
              O.normalize(O.fold1d(O.sfs1d(p, idx, 2, ocfg))))
        recs = F.snp_records(p, args[0], ocfg, lambda _c: bg)
        return post.bysnp_scan(recs, p, args[0], False, True)
    if fn in ("T2D_scan", "T1D_scan"):
        # the drop-in's host side (stream rebuild, packing) with oracle-made records
        from sfs2d.pack import last_key_index, pack_snp_dict, shadow_chrom_starts
        data, bg, extra = gu.t12_inputs(p, cfgd, fn, args)
        ws = extra[0]
        if fn == "T2D_scan":
            q = shadow_chrom_starts(p, last_key_index(data, p), ws, cfgd.get("start_position"),
                                    cfgd.get("end_position"))
            qcfg = O.Cfg(cfgd["n1p"], cfgd["n2p"], cfgd.get("variant_type"), cfgd.get("fold", True))
            n2 = 2 * cfgd["n2p"] + 1
            g = np.array([bg[(k // n2, k % n2)] for k in range(len(bg))]).reshape(-1, n2)
            ones = np.ones(cfgd["n1p"] + 1), np.ones(cfgd["n2p"] + 1)
            recs = F.bp_records(q, ws, qcfg, lambda _c: (g,) + ones)
            return post.single_stat_scan(recs, q, ws, post.num_slots(recs), 2, "T2D")
        pop, npop = extra[1], extra[2]
        q = (pack_snp_dict(data, pop, pop) if isinstance(data, dict) else p).single_pop(pop)
        qcfg = O.Cfg(npop, npop, cfgd.get("variant_type"), False, cfgd.get("start_position"), cfgd.get("end_position"))
        g1 = np.array([bg[k] for k in range(len(bg))])
        recs = F.bp_records(q, ws, qcfg, lambda _c: (np.ones((2 * npop + 1, 2 * npop + 1)), g1, np.ones(npop + 1)))
        return post.single_stat_scan(recs, q, ws, post.num_slots(recs), 1, "T1D")
    raise KeyError(fn)


_G = gu.Golden()
_CASES = [(n, i) for n in _G.cases() if n != "chr1" for i, c in enumerate(_G.calls(n))
          if c["fn"] != "sims_process_window"]


@pytest.mark.parametrize("name,i", _CASES, ids=[f"{n}-{i}" for n, i in _CASES])
def test_post_pass_vs_reference(golden, name, i):
    call = golden.calls(name)[i]
    p = golden.packed(name)
    ok, out, stdout = gu.run_capture(_post_call, p, golden.cfg(name), call["fn"], call["args"])
    ref = call["out"]
    if not ref["ok"]:
        assert not ok
        assert type(out).__name__ == ref["error"] and str(out) == ref["message"]
        return
    assert ok, repr(out)
    errs = gu.compare_results(out, gu.decode_results(ref["results"]))
    assert not errs, errs[:10]
    assert stdout == ref["stdout"]


def test_post_pass_chr1_20kb(golden):
    call = golden.calls("chr1")[0]
    assert call["fn"] == "combined_scan" and call["args"] == [20000]
    out = _post_call(golden.packed("chr1"), golden.cfg("chr1"), "combined_scan", [20000])
    errs = gu.compare_results(out, gu.decode_results(call["out"]["results"]))
    assert not errs, errs[:10]
