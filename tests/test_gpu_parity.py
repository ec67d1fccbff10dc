"""GPU parity: the drop-in modules (HIP kernels through the C ABI) against the reference's
golden outputs (tests/golden, produced by the reference's own functions) and against the
oracle's per-window records.  Integer counts bit-exact; float statistics within 1e-10 relative
(golden_util.close); exact 0.0 / inf / NaN / None identity."""
import numpy as np
import pytest

import golden_util as gu
from oracle import sfs_oracle as O

pytestmark = pytest.mark.gpu

_G = gu.Golden()


def _class_obj(cfgd):
    import twoDSFS_class as T
    return T.LikelihoodInference_jointSFS(None, None, start_position=cfgd.get("start_position"),
                                          end_position=cfgd.get("end_position"), pop1=cfgd["pop1"],
                                          pop2=cfgd["pop2"], pop1_size=cfgd["n1p"], pop2_size=cfgd["n2p"],
                                          variant_type=cfgd.get("variant_type"), fold=cfgd.get("fold", True))


def _gpu_call(obj, p, fn, args):
    if fn == "scan_precomputed_BG":
        d = p  # PackedSNPs accepted by every method
        bg2 = obj.normalize_2d_sfs(obj.calculate_2d_sfs(d))
        bg1 = obj.normalize_1d_sfs(obj.fold_1d_sfs(obj.calculate_1d_sfs(
            d, obj.pop1, obj.pop1_size, obj.start_position, obj.end_position, obj.variant_type)))
        bg1b = obj.normalize_1d_sfs(obj.fold_1d_sfs(obj.calculate_1d_sfs(
            d, obj.pop2, obj.pop2_size, obj.start_position, obj.end_position, obj.variant_type)))
        return obj.scan_precomputed_BG(p, args[0], bg2, bg1, bg1b)
    if fn in ("T2D_scan", "T1D_scan"):
        cfgd = dict(n1p=obj.pop1_size, n2p=obj.pop2_size, variant_type=obj.variant_type, fold=obj.fold,
                    start_position=obj.start_position, end_position=obj.end_position)
        data, bg, extra = gu.t12_inputs(p, cfgd, fn, args)
        return getattr(obj, fn)(data, bg, *extra)
    return getattr(obj, fn)(p, *args)


def _cases():
    out = []
    for name in _G.cases():
        for i, c in enumerate(_G.calls(name)):
            if c["fn"] != "sims_process_window":
                out.append((name, i))
    return out


@pytest.mark.parametrize("name,i", _cases(), ids=[f"{n}-{i}" for n, i in _cases()])
def test_dropin_class_vs_reference(golden, name, i):
    call = golden.calls(name)[i]
    p = golden.packed(name)
    cfgd = golden.cfg(name)
    obj = _class_obj(cfgd)
    ok, out, stdout = gu.run_capture(_gpu_call, obj, p, call["fn"], call["args"])
    ref = call["out"]
    if not ref["ok"]:
        assert not ok, f"reference raised {ref['error']}, GPU path returned"
        assert type(out).__name__ == ref["error"], repr(out)
        assert str(out) == ref["message"]
        return
    assert ok, f"GPU path raised {out!r}"
    errs = gu.compare_results(out, gu.decode_results(ref["results"]))
    assert not errs, errs[:10]
    assert stdout == ref["stdout"]


@pytest.mark.parametrize("tag", ["sims_n10", "sims_n100"])
def test_dropin_sims_vs_reference(golden, tag):
    import sims_scan as S
    call = golden.calls(tag)[0]
    rep = golden.packed(tag)
    bgd = golden.packed(f"{tag}_bgdata")
    n = golden.cfg(tag)["n1p"]
    bg2 = S.calculate_2d_sfs(bgd, "p1", "p2", n, n, start_position=0, end_position=500000, variant_type=None)
    bg1 = S.calculate_1d_sfs(bgd, "p1", n, start_position=0, end_position=500000, variant_type=None)
    bg1b = S.calculate_1d_sfs(bgd, "p2", n, start_position=0, end_position=500000, variant_type=None)
    gb = golden.npz(f"{tag}_bg.npz")
    assert np.array_equal(np.array([[bg2[(i, j)] for j in range(2 * n + 1)] for i in range(2 * n + 1)]), gb["bg2d"])
    assert np.array_equal(np.array([bg1[k] for k in range(2 * n + 1)]), gb["bg1a"])
    out = S.process_window(rep, bg2, bg1, bg1b, 500000, "p1", "p2", n, n, None, None, None)
    errs = gu.compare_results(out, gu.decode_results(call["out"]["results"]))
    assert not errs, errs[:10]


def test_bg_hist_bitexact_chr1(golden):
    from sfs2d.engine import Engine, ScanConfig
    p = golden.packed("chr1")
    eng = Engine.get(0)
    dev = eng.upload(p)
    h2, u1, u2 = eng.bg_hist(dev, ScanConfig(n1p=18, n2p=14), 0)
    import twoDSFS_class as T
    g = golden.npz("chr1_bg.npz")
    assert np.array_equal(h2, g["bg2d"])
    assert np.array_equal(T._fold_counts(u1), g["bg1a"])
    assert np.array_equal(T._fold_counts(u2), g["bg1b"])


def _records_vs_oracle(p, cfg_scan, ocfg, wins, bg_of, guards=True, bg=None):
    from sfs2d import _lib as L
    from sfs2d.engine import Engine
    eng = Engine.get(0)
    dev = eng.upload(p)
    recs = eng.scan(dev, cfg_scan, bg=bg)
    body = recs[(recs["flags"] & (L.W_EMPTY | L.W_EXTRA)) == 0]
    ref = O.window_records(p, wins, ocfg, bg_of, guards)
    assert len(body) == len(ref)
    for r, o in zip(body, ref):
        for f, g in (("snp_count", "snp_count"), ("n2", "N2"), ("n2_all", "N2_all"), ("n1a", "N1a"), ("n1b", "N1b")):
            assert int(r[f]) == o[g], (f, int(r[f]), o[g])
        for f, g in (("t2d", "T2D"), ("t1d_p1", "T1D_p1"), ("t1d_p2", "T1D_p2")):
            if o[g] is not None:
                assert gu.close(float(r[f]), o[g]), (f, float(r[f]), o[g])
    return body


@pytest.mark.parametrize("n1p,n2p,ws", [(25, 25, 20000), (18, 14, 7000), (50, 50, 20000), (100, 75, 100000),
                                          (3, 2, 500), (25, 25, 500000), (40, 40, 20000), (44, 30, 20000),
                                          (31, 31, 20000), (32, 31, 20000), (60, 8, 20000), (8, 60, 20000),
                                          (70, 5, 20000)])
def test_records_per_chrom_bp(n1p, n2p, ws):
    """(40 x 40, 44 x 30: grids under the small-grid limit whose k_scan_w workgroup does not fit the
    LDS take the large-grid kernels.  31 x 31: the largest populations whose folded 1D bins 0..n_p k_scan_w
    reads on half a wave each; 32 x 31, 60 x 8, 8 x 60: its one-bin-per-lane path, bins 0 and n_p of a
    population in different lanes; 70 x 5: bin n_p in the second register.)"""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [4000, 2500, 1], n1p, n2p, seed=n1p * 7 + ws)
    ocfg = O.Cfg(n1p, n2p)
    bgs = O.chrom_backgrounds(p, ocfg)
    _records_vs_oracle(p, ScanConfig(n1p=n1p, n2p=n2p, window=ws), ocfg, O.bp_windows(p, ws), lambda c: bgs[c])


@pytest.mark.parametrize("S", [1, 64, 500, 4096])
def test_records_per_chrom_snps(S):
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [5000, 3333], 25, 25, seed=S)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    wins, _ = O.snp_windows(p, S)
    _records_vs_oracle(p, ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=S), ocfg, wins,
                       lambda c: bgs[c])


def test_records_large_histogram_with_fst():
    """pop_size 95 / 95 with Fst: the background histogram (148 KB) no longer fits the LDS beside the
    Fst k_prep's static window sums; the plan must still run (global-atomic histogram) and match the
    oracle's records."""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [3000, 1700], 95, 95, seed=9595)
    ocfg = O.Cfg(95, 95)
    bgs = O.chrom_backgrounds(p, ocfg)
    wins, _ = O.snp_windows(p, 400)
    _records_vs_oracle(p, ScanConfig(n1p=95, n2p=95, window_mode=L.WINDOW_SNPS, window=400, fst=True), ocfg, wins,
                       lambda c: bgs[c])


def test_config2_full_size_self_consistency():
    """BASELINE config 2 (1e6 SNPs, n1=n2=50 haploid, 20 kb): every window's counts partition the
    stream, the 2D/1D totals equal the background totals, and a 200-window sample matches the
    oracle."""
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(1, 1_000_000, 25, 25, seed=12345)
    eng = Engine.get(0)
    dev = eng.upload(p)
    recs = eng.scan(dev, ScanConfig(n1p=25, n2p=25, window=20000))
    body = recs[(recs["flags"] & L.W_EMPTY) == 0]
    assert int(body["snp_count"].sum()) == p.n
    assert np.all(body["begin"][1:] == body["end"][:-1])
    h2, u1, u2 = eng.bg_hist(dev, ScanConfig(n1p=25, n2p=25), 0)
    assert int(body["n2"].sum()) == int(h2.ravel()[1:-1].sum())
    ocfg = O.Cfg(25, 25)
    bg = O.chrom_backgrounds(p, ocfg)[0]
    wins = O.bp_windows(p, 20000)
    assert len(wins) == len(body)
    idx = np.linspace(0, len(wins) - 1, 200).astype(int)
    ref = O.window_records(p, [wins[i] for i in idx], ocfg, lambda c: bg)
    for i, o in zip(idx, ref):
        r = body[i]
        assert int(r["n2"]) == o["N2"] and int(r["n1a"]) == o["N1a"] and int(r["n1b"]) == o["N1b"]
        assert gu.close(float(r["t2d"]), o["T2D"]) and gu.close(float(r["t1d_p1"]), o["T1D_p1"])
        assert gu.close(float(r["t1d_p2"]), o["T1D_p2"])


def test_plan_replay_is_deterministic():
    """Self-cleaning state (slot table, background replicas, LDS) across repeated runs."""
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [20000, 7000], 25, 25, seed=9)
    eng = Engine.get(0)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, prev_extra=True))
    outs = []
    for _ in range(3):
        pl.run()
        pl.check()
        outs.append(pl.read())
    assert outs[0].tobytes() == outs[1].tobytes() == outs[2].tobytes()
    pl.close()


@pytest.mark.parametrize("fst,nplans", [(False, 3), (True, 3), (True, 2)])
def test_run_streams_overlapped_plans(fst, nplans):
    """sfs2d_plan_run_streams: passes round-robin over plans on their own HIP streams (overlapping; the
    second stream's first pass waits for the first pass's k_prep) write the same records and Fst as one
    plan run alone; argument errors are reported."""
    import torch
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, Plan, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(1, 200000, 25, 25, seed=4242)
    eng = Engine.get(0)
    dev = eng.upload(p)
    cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=fst)
    ref = eng.plan(dev, cfg)
    ref.run()
    ref.check()
    want = ref.read()
    want_f = ref.read_fst() if fst else None
    plans = [eng.plan(dev, cfg) for _ in range(nplans)]
    streams = [torch.cuda.Stream(device=0).cuda_stream for _ in range(nplans)]
    outs = [torch.zeros((plans[0].nrec, 64), dtype=torch.uint8, device="cuda:0") for _ in range(nplans)]
    Plan.run_streams(plans, streams, nplans * 5 + 1, [o.data_ptr() for o in outs])
    torch.cuda.synchronize()
    for k, q in enumerate(plans):
        q.check()
        got = np.frombuffer(outs[k].cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
        assert got.tobytes() == want.tobytes(), k
        if fst:
            assert np.array_equal(q.read_fst(), want_f, equal_nan=True), k
    with pytest.raises(L.Sfs2dError):
        Plan.run_streams([plans[0], plans[0]], streams[:2], 2)
    for q in plans + [ref]:
        q.close()
    dev.close()


def test_graph_replay_snp_windows_large_grid():
    """Config 5's bench shape replayed as HIP graphs (bench.py config5_snpwin): 500-SNP windows at pop
    100/75 (201 x 151 grid, k_scan_gw), per-chromosome backgrounds, 4 plans on 4 streams -- every
    replay's records byte-equal to one plan run alone (whose SNP-window records the oracle pins in
    test_large_grid_kernels / the bySNPs goldens)."""
    import torch
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, Plan, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [40000, 25000], 100, 75, seed=6262)
    eng = Engine.get(0)
    dev = eng.upload(p)
    cfg = ScanConfig(n1p=100, n2p=75, window_mode=L.WINDOW_SNPS, window=500)
    ref = eng.plan(dev, cfg)
    ref.run()
    ref.check()
    want = ref.read()
    plans = [eng.plan(dev, cfg) for _ in range(4)]
    streams = [torch.cuda.Stream(device=0).cuda_stream for _ in range(4)]
    outs = [torch.zeros((plans[0].nrec, 64), dtype=torch.uint8, device="cuda:0") for _ in range(4)]
    g = Plan.graph(plans, streams, 16, [o.data_ptr() for o in outs])
    for rep in range(2):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        g.launch(rep + 1)
        torch.cuda.synchronize()
        for k, q in enumerate(plans):
            q.check()
            got = np.frombuffer(outs[k].cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
            assert got.tobytes() == want.tobytes(), (rep, k)
    g.close()
    for q in plans + [ref]:
        q.close()
    dev.close()


@pytest.mark.parametrize("fst,nplans", [(True, 3), (False, 2), (True, 1)])
def test_graph_replay(fst, nplans):
    """sfs2d_graph_*: a run_streams sequence captured into a HIP graph and replayed writes the same
    records and Fst as one plan run alone, every replay (outputs cleared in between); a capture of an
    odd number of runs per plan, or with timing on, is refused, and so is a replay after a plan ran an
    odd number of times since the capture (its buffer parity changed); an even number brings it back."""
    import torch
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, Plan, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [200000, 60000], 25, 25, seed=5151)
    eng = Engine.get(0)
    dev = eng.upload(p)
    cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=fst)
    ref = eng.plan(dev, cfg)
    ref.run()
    ref.check()
    want = ref.read()
    want_f = ref.read_fst() if fst else None
    plans = [eng.plan(dev, cfg) for _ in range(nplans)]
    streams = [torch.cuda.Stream(device=0).cuda_stream for _ in range(nplans)]
    outs = [torch.zeros((plans[0].nrec, 64), dtype=torch.uint8, device="cuda:0") for _ in range(nplans)]
    optrs = [o.data_ptr() for o in outs]
    with pytest.raises(L.Sfs2dError):
        Plan.graph(plans, streams, 2 * nplans + nplans, optrs)
    plans[0].set_timing(4)
    with pytest.raises(L.Sfs2dError):
        Plan.graph(plans, streams, 2 * nplans, optrs)
    plans[0].set_timing(0)
    g = Plan.graph(plans, streams, 4 * nplans, optrs)

    def check_all():
        torch.cuda.synchronize()
        for k, q in enumerate(plans):
            q.check()
            got = np.frombuffer(outs[k].cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
            assert got.tobytes() == want.tobytes(), k
            if fst:
                assert np.array_equal(q.read_fst(), want_f, equal_nan=True), k

    for rep in range(3):
        for o in outs:
            o.zero_()
        torch.cuda.synchronize()
        g.launch(rep + 1)
        check_all()
    plans[0].run(optrs[0])
    with pytest.raises(L.Sfs2dError):
        g.launch()
    plans[0].run(optrs[0])
    for o in outs:
        o.zero_()
    torch.cuda.synchronize()
    g.launch(2)
    check_all()
    g.close()
    for q in plans + [ref]:
        q.close()
    dev.close()


def test_run_streams_none_is_the_engine_stream():
    """Plan.run_streams with None entries enqueues on the engine's current stream (its own stream by
    default, sfs2d_ctx_get_stream), so read() -- which synchronises that stream only -- returns the
    finished runs' records without any other synchronisation; 0 is the HIP null stream."""
    from sfs2d.engine import Engine, Plan, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [300000, 200000], 25, 25, seed=99)
    eng = Engine.get(0)
    assert eng.stream_handle() != 0   # the ctx's own non-blocking stream
    dev = eng.upload(p)
    cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=True)
    ref = eng.plan(dev, cfg)
    ref.run()
    want = ref.read()
    plans = [eng.plan(dev, cfg) for _ in range(2)]
    Plan.run_streams(plans, [None, None], 6)
    for q in plans:
        assert q.read().tobytes() == want.tobytes()
        q.check()
    prev = eng.set_stream(0)
    try:
        assert eng.stream_handle() == 0
        Plan.run_streams(plans, [None, 0], 4)
        for q in plans:
            assert q.read().tobytes() == want.tobytes()
    finally:
        eng.set_stream(prev)
    for q in plans + [ref]:
        q.close()
    dev.close()


def test_fst_out_buffers_per_run():
    """sfs2d_plan_set_fst_out: consecutive runs of one plan write their Fst columns into caller buffers
    (bench.py's per-pass gathered loop), equal to the plan-owned buffer's values; None restores it."""
    import torch
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [200000, 90000], 25, 25, seed=31)
    eng = Engine.get(0)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
    pl.run()
    want = pl.read_fst()
    bufs = [torch.full((len(want),), -1.0, dtype=torch.float64, device="cuda:0") for _ in range(2)]
    prev = eng.set_stream(torch.cuda.current_stream().cuda_stream)
    try:
        for b in bufs:
            pl.set_fst_out(b.data_ptr())
            pl.run()
        torch.cuda.synchronize()
        for b in bufs:
            assert np.array_equal(b.cpu().numpy(), want, equal_nan=True)
        pl.set_fst_out(None)
        pl.run()
        assert np.array_equal(pl.read_fst(), want, equal_nan=True)
    finally:
        eng.set_stream(prev)
    pl.close()
    dev.close()


def test_key_error_on_counts_above_sample_size():
    import twoDSFS_class as T
    d = {"c-1": {"calls": {"uv": (0, 3), "bv": (2, 0)}, "annotation": "x"},
         "c-5": {"calls": {"uv": (1, 1), "bv": (1, 1)}, "annotation": "x"}}
    obj = T.LikelihoodInference_jointSFS(None, None, pop1_size=1, pop2_size=1)
    with pytest.raises(KeyError):
        obj.combined_scan(d, 100)


def _bad_count_dict():
    """Two chromosomes (pop_size 2: 4 alleles per population); chromosome "b" holds one SNP whose pop-1
    alt count (5) exceeds 2 * pop_size."""
    d = {}
    for c in ("a", "b"):
        for i in range(1, 60):
            a, b = i % 5, (i // 2) % 5
            d[f"{c}-{i * 3}"] = {"calls": {"uv": (4 - a, a), "bv": (4 - b, b)}, "annotation": "x"}
    d["b-50"] = {"calls": {"uv": (0, 5), "bv": (1, 1)}, "annotation": "x"}
    return d


@pytest.mark.parametrize("driver", ["precomputed", "chooseChr", "chooseChr_bySNPs", "perChr_bySNPs"])
def test_key_error_with_supplied_background(driver):
    """Counts above 2 * pop_size raise KeyError (calculate_1d_sfs, twoDSFS_class.py:433) also when the
    background is supplied: those plans run no k_prep pass over the counts, so a data set whose called
    counts exceed the grid takes the bins pipeline, whose k_prep reports the SNP."""
    import twoDSFS_class as T
    d = _bad_count_dict()
    obj = T.LikelihoodInference_jointSFS(None, None, pop1_size=2, pop2_size=2)
    good = {k: v for k, v in d.items() if k.startswith("a-")}
    bg2 = obj.calculate_2d_sfs(good)
    bg1 = obj.fold_1d_sfs(obj.calculate_1d_sfs(good, "uv", 2, None, None, None))
    bg1b = obj.fold_1d_sfs(obj.calculate_1d_sfs(good, "bv", 2, None, None, None))
    with pytest.raises(KeyError):
        if driver == "precomputed":
            obj.scan_precomputed_BG(d, 100, bg2, bg1, bg1b)
        elif driver == "chooseChr":
            obj.scan_chooseChr(d, 100, "a")
        elif driver == "chooseChr_bySNPs":
            obj.scan_chooseChr_bySNPs(d, 5, "a")
        else:
            obj.scan_perChr_bySNPs(d, 5)
    # the same calls on the clean chromosome run (a counts plan: its called counts are within the grid)
    from sfs2d.pack import pack_snp_dict
    q = pack_snp_dict(good)
    ocfg = O.Cfg(2, 2)
    r = obj.scan_precomputed_BG(good, 100, bg2, bg1, bg1b)
    assert list(r) == ["a 1-100", "a 101-200"] and all(v["T2D"] is not None for v in r.values())
    got = obj.scan_chooseChr_bySNPs(good, 5, "a")
    want = O.scan_chooseChr_bySNPs(q, 5, "a", ocfg)
    assert list(got) == list(want) and len(got) > 5


def test_dense_primitives_vs_oracle(golden):
    p = golden.packed("synth_n50")
    import twoDSFS_class as T
    obj = T.LikelihoodInference_jointSFS(None, None, pop1="p1", pop2="p2", pop1_size=25, pop2_size=25)
    d = p.subset_chroms([0])
    bg = obj.calculate_2d_sfs(d)
    win = p.subset_chroms([2])
    fg = obj.calculate_2d_sfs(win)
    ocfg = O.Cfg(25, 25)
    g_fg = O.sfs2d(win, np.arange(win.n), ocfg)
    g_bg = O.sfs2d(d, np.arange(d.n), ocfg)
    assert fg == {(i, j): int(g_fg[i, j]) for i in range(51) for j in range(51)}
    assert gu.close(obj.calculate_likelihood_2D(fg, bg), O.clr2d(g_fg, g_bg))
    f1 = obj.fold_1d_sfs(obj.calculate_1d_sfs(win, "p1", 25, None, None, None))
    b1 = obj.fold_1d_sfs(obj.calculate_1d_sfs(d, "p1", 25, None, None, None))
    o1 = O.clr1d(O.fold1d(O.sfs1d(win, np.arange(win.n), 1, ocfg)), O.fold1d(O.sfs1d(d, np.arange(d.n), 1, ocfg)))
    assert gu.close(obj.calculate_likelihood_1D(f1, b1), o1)


def test_sharded_combined_scan_world1_matches_class():
    """sfs2d.dist end to end on one GPU (gloo group of one): shard, scan, gather, merge, post-pass."""
    import os
    import torch.distributed as dist
    import twoDSFS_class as T
    from sfs2d import dist as D
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [6000, 2500, 1], 25, 25, seed=21)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        got = D.combined_scan_sharded(p, 20000, 25, 25, rank=0, world=1)
    finally:
        dist.destroy_process_group()
    obj = T.LikelihoodInference_jointSFS(None, None, pop1="p1", pop2="p2", pop1_size=25, pop2_size=25)
    ref = obj.combined_scan(p, 20000)
    errs = gu.compare_results(got, ref)
    assert not errs, errs[:10]


def test_rank_overflow_big_bins_bp():
    """Bins holding more than the LDS D-table's 511 ranks (k_scan_w adds F(x) - F(511) per bin)."""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.pack import pack_counts
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [4000, 2600], 25, 25, seed=77)
    rng = np.random.default_rng(3)
    hot = rng.random(p.n) < 0.6            # 60% of the SNPs share the bin (1, 0)
    a1 = np.where(hot, 1, p.alt1); r1 = np.where(hot, 49, p.ref1)
    a2 = np.where(hot, 0, p.alt2); r2 = np.where(hot, 50, p.ref2)
    p.counts = pack_counts(r1, a1, r2, a2)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    for ws in (10_000_000, 100_000):
        _records_vs_oracle(p, ScanConfig(n1p=25, n2p=25, window=ws), ocfg, O.bp_windows(p, ws), lambda c: bgs[c])


def test_snp_windows_of_65536_plus_take_exact_path():
    """Windows of >= 65536 SNPs: 32-bit 2D bins and the exact evaluation (fused table view)."""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(1, 150_000, 25, 25, seed=8)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    wins, _ = O.snp_windows(p, 70000)
    _records_vs_oracle(p, ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=70000), ocfg, wins,
                       lambda c: bgs[c])


def _fst_close(a, b):
    if b is None:
        return np.isnan(a)
    return abs(a - b) <= 1e-12 + 1e-10 * abs(b)


@pytest.mark.parametrize("n1p,n2p,mode,ws", [(25, 25, "bp", 20000), (18, 14, "bp", 7000), (25, 25, "snps", 500),
                                             (100, 75, "snps", 500), (95, 95, "snps", 400), (95, 95, "bp", 20000)])
def test_fst_vs_oracle(n1p, n2p, mode, ws):
    """Hudson Fst per window (k_scan_w fast path, k_scan_g for the 201x151 grid) against
    oracle.window_fst (parity of Fst itself is unpinned: the reference has no Fst).  95 x 95: a
    background histogram (148 KB) that fits the LDS alone but not beside the Fst k_prep's static
    sums, which then takes the global-atomic histogram."""
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [6000, 2500], n1p, n2p, seed=n1p + ws)
    ocfg = O.Cfg(n1p, n2p)
    eng = Engine.get(0)
    dev = eng.upload(p)
    if mode == "bp":
        cfg = ScanConfig(n1p=n1p, n2p=n2p, window=ws, fst=True)
        wins = [(b, e) for (c, s, b, e) in O.bp_windows(p, ws)]
    else:
        cfg = ScanConfig(n1p=n1p, n2p=n2p, window_mode=L.WINDOW_SNPS, window=ws, fst=True)
        wins = [(w[3], w[4]) for w in O.snp_windows(p, ws)[0]]
    pl = eng.plan(dev, cfg)
    pl.run()
    pl.check()
    recs = pl.read()
    fst = pl.read_fst()
    live = (recs["flags"][: len(fst)] & L.W_EMPTY) == 0
    assert np.all(np.isnan(fst[~live]))
    got = fst[live]
    assert len(got) == len(wins)
    for g, (b, e) in zip(got, wins):
        assert _fst_close(float(g), O.window_fst(p, np.arange(b, e), ocfg)), (g, b, e)
    pl.close()


@pytest.mark.parametrize("wgs", ["3", "17"])
def test_dynamic_window_pools(monkeypatch, wgs):
    """k_scan_w with few workgroups: most windows come from the per-chromosome pool counters
    (both counter parities, over repeated runs) and every window is still scanned exactly once."""
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    monkeypatch.setenv("SFS2D_WGS", wgs)
    p = synth_genome(3, [12000, 6000, 5], 25, 25, seed=int(wgs))
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    for mode, ws in ((L.WINDOW_SNPS, 16), (L.WINDOW_BP, 3000)):
        cfg = ScanConfig(n1p=25, n2p=25, window_mode=mode, window=ws)
        wins = O.snp_windows(p, ws)[0] if mode == L.WINDOW_SNPS else O.bp_windows(p, ws)
        _records_vs_oracle(p, cfg, ocfg, wins, lambda c: bgs[c])
        eng = Engine.get(0)
        dev = eng.upload(p)
        pl = eng.plan(dev, cfg)
        outs = []
        for _ in range(3):
            pl.run()
            outs.append(pl.read().tobytes())
        assert outs[0] == outs[1] == outs[2]


@pytest.mark.parametrize("gw", ["0", "1"])
@pytest.mark.parametrize("n1p,n2p", [(50, 50), (100, 75)])
def test_large_grid_kernels(monkeypatch, gw, n1p, n2p):
    """Grids > 8192 bins through each large-grid kernel, forced on both grid sizes (by default
    both take k_scan_gw, a wavefront per window with the tables read from L2; k_scan_g, a
    workgroup per window, is kept for grids leaving one such wavefront per CU): records of fixed-bp
    and SNP-count windows over many chromosomes (k_scan_gw's several workgroups per chromosome),
    Fst, and repeated runs."""
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    monkeypatch.setenv("SFS2D_GW", gw)
    p = synth_genome(9, [700 + 311 * i for i in range(8)] + [3], n1p, n2p, seed=n1p * 3 + int(gw))
    ocfg = O.Cfg(n1p, n2p)
    bgs = O.chrom_backgrounds(p, ocfg)
    for mode, ws in ((L.WINDOW_BP, 30000), (L.WINDOW_SNPS, 90)):
        cfg = ScanConfig(n1p=n1p, n2p=n2p, window_mode=mode, window=ws)
        wins = O.snp_windows(p, ws)[0] if mode == L.WINDOW_SNPS else O.bp_windows(p, ws)
        _records_vs_oracle(p, cfg, ocfg, wins, lambda c: bgs[c])
    eng = Engine.get(0)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=n1p, n2p=n2p, window=30000, fst=True))
    last = [int(p.pos[p.chrom_off[c + 1] - 1]) for c in range(p.nchrom)]
    nslots = [(max(x, 1) - 1) // 30000 + 1 for x in last]   # fixed-bp slots per chromosome
    g_threads = 256 * sum((n + 1) // 2 for n in nslots)   # k_scan_g: two windows per workgroup
    assert (pl.grids()[1] == g_threads) == (gw == "0")
    outs = []
    for _ in range(3):
        pl.run()
        pl.check()
        outs.append((pl.read(), pl.read_fst()))
    recs, fst = outs[0]
    live = (recs["flags"][: len(fst)] & L.W_EMPTY) == 0
    got = fst[live]
    wins = [(b, e) for (c, s, b, e) in O.bp_windows(p, 30000)]
    assert len(got) == len(wins)
    for g, (b, e) in zip(got, wins):
        assert _fst_close(float(g), O.window_fst(p, np.arange(b, e), ocfg)), (g, b, e)
    for r, f in outs[1:]:
        assert np.array_equal(r["snp_count"], recs["snp_count"]) and np.array_equal(f, fst, equal_nan=True)
        for k in ("t2d", "t1d_p1", "t1d_p2"):
            a, b = r[k].astype(float), recs[k].astype(float)
            assert np.allclose(a, b, rtol=1e-12, atol=1e-12, equal_nan=True)
    pl.close()


@pytest.mark.parametrize("n1p,n2p", [(50, 50), (100, 75)])
def test_large_grid_u8_bins_wrap(n1p, n2p):
    """k_scan_gw counts 2D bins in bytes: windows with >= 256 SNPs in one bin wrap a byte and are
    re-evaluated exactly on global-memory histograms (many waves at once: every window of the
    first chromosome wraps).  Records of fixed-bp and SNP-count windows against the oracle."""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.pack import PackedSNPs, pack_counts
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [9000, 4000, 700], n1p, n2p, seed=77)
    r1, a1 = (p.counts & 0xff).astype(np.int64), ((p.counts >> 8) & 0xff).astype(np.int64)
    r2, a2 = ((p.counts >> 16) & 0xff).astype(np.int64), (p.counts >> 24).astype(np.int64)
    same = np.zeros(p.n, bool)
    same[: p.chrom_off[1]] = True                                   # chromosome 0: one 2D bin only
    same[p.chrom_off[1]: p.chrom_off[1] + 1500] = np.arange(1500) % 3 != 0   # chromosome 1: 2 in 3
    r1 = np.where(same, 2 * n1p - 1, r1); a1 = np.where(same, 1, a1)
    r2 = np.where(same, 2 * n2p - 2, r2); a2 = np.where(same, 2, a2)
    q = PackedSNPs(pack_counts(r1, a1, r2, a2), p.pos, p.chrom_off, p.chrom_names, p.ann_id, p.ann_names)
    ocfg = O.Cfg(n1p, n2p)
    bgs = O.chrom_backgrounds(q, ocfg)
    for mode, ws in ((L.WINDOW_BP, 60000), (L.WINDOW_SNPS, 700)):
        wins = O.snp_windows(q, ws)[0] if mode == L.WINDOW_SNPS else O.bp_windows(q, ws)
        _records_vs_oracle(q, ScanConfig(n1p=n1p, n2p=n2p, window_mode=mode, window=ws), ocfg, wins,
                           lambda c: bgs[c])


@pytest.mark.parametrize("n1p,n2p", [(50, 50), (100, 75)])
def test_large_grid_bins_past_63(n1p, n2p):
    """k_scan_gw takes D(r) for ranks r < 63 from lane shuffles and adds F(x) - F(63) at the window's
    end for each bin holding x > 63 SNPs (no wrap: x < 255): windows with one bin holding ~50 to ~100
    SNPs (every 4th / 6th / 7th SNP forced into one bin), fixed-bp and SNP-count windows, against the
    oracle."""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.pack import PackedSNPs, pack_counts
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [6000, 3000, 2500], n1p, n2p, seed=63)
    r1, a1 = (p.counts & 0xff).astype(np.int64), ((p.counts >> 8) & 0xff).astype(np.int64)
    r2, a2 = ((p.counts >> 16) & 0xff).astype(np.int64), (p.counts >> 24).astype(np.int64)
    i = np.arange(p.n)
    c = np.searchsorted(p.chrom_off, i, side="right") - 1
    same = (i - p.chrom_off[c]) % np.array([4, 6, 7])[c] == 0
    r1 = np.where(same, 2 * n1p - 3, r1); a1 = np.where(same, 3, a1)
    r2 = np.where(same, 2 * n2p - 1, r2); a2 = np.where(same, 1, a2)
    q = PackedSNPs(pack_counts(r1, a1, r2, a2), p.pos, p.chrom_off, p.chrom_names, p.ann_id, p.ann_names)
    ocfg = O.Cfg(n1p, n2p)
    bgs = O.chrom_backgrounds(q, ocfg)
    for mode, ws in ((L.WINDOW_BP, 20000), (L.WINDOW_SNPS, 400)):
        wins = O.snp_windows(q, ws)[0] if mode == L.WINDOW_SNPS else O.bp_windows(q, ws)
        _records_vs_oracle(q, ScanConfig(n1p=n1p, n2p=n2p, window_mode=mode, window=ws), ocfg, wins,
                           lambda c: bgs[c])


@pytest.mark.parametrize("gw", ["0", "1"])
def test_largest_grid(monkeypatch, gw):
    """The largest grid the u8 allele counts allow (pop_size 127: 255 x 255 = 65,025 bins, 16-bit 2D
    keys, 7-bit folded 1D keys): both large-grid kernels against the oracle."""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    monkeypatch.setenv("SFS2D_GW", gw)
    p = synth_genome(2, [5000, 1200], 127, 127, seed=127)
    ocfg = O.Cfg(127, 127)
    bgs = O.chrom_backgrounds(p, ocfg)
    for mode, ws in ((L.WINDOW_BP, 50000), (L.WINDOW_SNPS, 300)):
        wins = O.snp_windows(p, ws)[0] if mode == L.WINDOW_SNPS else O.bp_windows(p, ws)
        _records_vs_oracle(p, ScanConfig(n1p=127, n2p=127, window_mode=mode, window=ws), ocfg, wins,
                           lambda c: bgs[c])


def test_called_counts_above_sample_size_inside_long_tiles():
    """SNPs whose called allele count r + a exceeds 2 * pop_size without leaving the grid (no fold
    swap, so the 2D key is the alt count): the reference counts them; k_prep routes their steps
    through the exact classify, the rest of the tile through the fast path.  Records, Fst and the
    background histograms against the oracle."""
    import twoDSFS_class as T
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.pack import PackedSNPs, pack_counts
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [40000, 9000], 25, 25, seed=4242)
    r1, a1 = p.counts & 0xff, (p.counts >> 8) & 0xff
    r2, a2 = (p.counts >> 16) & 0xff, p.counts >> 24
    pick = (np.random.default_rng(3).random(p.n) < 0.004) & (a1 + a2 <= 50)
    q = PackedSNPs(pack_counts(np.where(pick, r1 + 7, r1), a1, r2, a2), p.pos, p.chrom_off, p.chrom_names,
                   p.ann_id, p.ann_names)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(q, ocfg)
    wins = O.bp_windows(q, 20000)
    _records_vs_oracle(q, ScanConfig(n1p=25, n2p=25, window=20000), ocfg, wins, lambda c: bgs[c])
    eng = Engine.get(0)
    dev = eng.upload(q)
    h2, u1, u2 = eng.bg_hist(dev, ScanConfig(n1p=25, n2p=25), 0)
    assert np.array_equal(np.asarray(h2), np.asarray(bgs[0][0]))
    assert np.array_equal(T._fold_counts(u1), np.asarray(bgs[0][1]))
    assert np.array_equal(T._fold_counts(u2), np.asarray(bgs[0][2]))
    pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
    pl.run()
    pl.check()
    recs = pl.read()
    fst = pl.read_fst()
    live = (recs["flags"][: len(fst)] & L.W_EMPTY) == 0
    got = fst[live]
    assert len(got) == len(wins)
    for g, (c, st, b, e) in list(zip(got, wins))[::7]:
        assert _fst_close(float(g), O.window_fst(q, np.arange(b, e), ocfg)), (g, b, e)
    pl.close()


@pytest.mark.parametrize("n1p,n2p,fold,ws", [(25, 25, True, 20000), (25, 25, False, 20000), (18, 14, True, 20000),
                                               (3, 2, True, 1000)])
def test_prep_joint_histogram(monkeypatch, n1p, n2p, fold, ws):
    """k_prep's joint (alt1, alt2) histogram (the common step of counts plans: one LDS atomic per SNP
    plus one per folded SNP, both 1D spectra from its margins at the tile's end) against the three
    atomics per SNP it replaced (SFS2D_JNT=0): byte-equal records and Fst, both against the oracle, on
    chromosomes long enough for many common steps (a step is 2,048 SNPs; edge steps and steps with
    over-called SNPs take the exact classify in the same tiles).  (The 7-bin grid scans 1 kb windows: at
    20 kb its T1D values of ~4e-4 are differences of ~2e3-sized sums, below 1e-10 relative in fp64 for
    any evaluation order, the oracle's included.)"""
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.pack import PackedSNPs, pack_counts
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [70001, 30000, 9], n1p, n2p, seed=n1p * 13 + n2p + fold)
    r1, a1 = p.counts & 0xff, (p.counts >> 8) & 0xff
    r2, a2 = (p.counts >> 16) & 0xff, p.counts >> 24
    pick = (np.random.default_rng(5).random(p.n) < 0.0005) & (a1 + a2 <= n1p + n2p)
    q = PackedSNPs(pack_counts(np.where(pick, r1 + 3, r1), a1, r2, a2), p.pos, p.chrom_off, p.chrom_names,
                   p.ann_id, p.ann_names)
    eng = Engine.get(0)
    dev = eng.upload(q)
    cfg = ScanConfig(n1p=n1p, n2p=n2p, fold=fold, window=ws, fst=True)
    out = {}
    for jnt in ("1", "0"):
        monkeypatch.setenv("SFS2D_JNT", jnt)
        pl = eng.plan(dev, cfg)
        pl.run()
        pl.check()
        out[jnt] = (pl.read(), pl.read_fst())
        pl.close()
    assert out["1"][0].tobytes() == out["0"][0].tobytes()
    assert out["1"][1].tobytes() == out["0"][1].tobytes()
    monkeypatch.setenv("SFS2D_JNT", "1")
    ocfg = O.Cfg(n1p, n2p, fold=fold)
    bgs = O.chrom_backgrounds(q, ocfg)
    _records_vs_oracle(q, cfg, ocfg, O.bp_windows(q, ws), lambda c: bgs[c])


def _overcall(p, n1p, n2p, frac, seed):
    """Copy of p with a fraction of SNPs made over-called in both populations: called counts r + a above
    2 pop_size with a1 + a2 > n1p + n2p (a joint fold) and r1 + r2 > n (a folded key outside the triangle
    x1 + x2 <= n); e.g. (60, 50, 45, 55) at pop 50/50.  Every alt count stays <= 2 pop_size (no KeyError)
    and every folded key inside the grid."""
    from sfs2d.pack import PackedSNPs, pack_counts
    n1, n2 = 2 * n1p, 2 * n2p
    rng = np.random.default_rng(seed)
    r1, a1 = (p.counts & 0xff).astype(np.int64), ((p.counts >> 8) & 0xff).astype(np.int64)
    r2, a2 = ((p.counts >> 16) & 0xff).astype(np.int64), (p.counts >> 24).astype(np.int64)
    pick = rng.random(p.n) < frac
    m = int(pick.sum())
    na1 = rng.integers(n1p, int(n1 * 0.7) + 1, m)          # a1 + a2 > n1p + n2p: the fold swaps
    na2 = rng.integers(n2p + 1, int(n2 * 0.7) + 1, m)
    nr1 = rng.integers(n1p + 1, n1 + 1, m)                 # r1 + r2 > n: outside the triangle
    nr2 = rng.integers(n2p - 4, n2 + 1, m)
    r1[pick], a1[pick], r2[pick], a2[pick] = nr1, na1, nr2, na2
    assert np.all(r1 <= 255) and np.all(r2 <= 255)
    q = PackedSNPs(pack_counts(r1, a1, r2, a2), p.pos, p.chrom_off, p.chrom_names, p.ann_id, p.ann_names)
    sel = pick & (a1 + a2 > n1p + n2p)
    assert np.any(sel & (r1 + r2 > n1)) and np.all(r1[sel] <= n1) and np.all(r2[sel] <= n2)
    return q


@pytest.mark.parametrize("n1p,n2p", [(50, 50), (100, 75)])
@pytest.mark.parametrize("fst", [False, True])
def test_large_grid_overcalled_snps_per_chrom(n1p, n2p, fst):
    """k_scan_gw's triangle histogram (folded square counts plans) is only exact
    while every called count is <= 2 pop_size; over-called SNPs (called count above 2 pop_size, folded
    key with x1 + x2 > n, e.g. (60, 50, 45, 55) at 50/50) are counted by the reference at their in-grid
    key (twoDSFS_class.py:198-217), so such data sets keep the full grid.  Per-chromosome backgrounds,
    fixed-bp and SNP-count windows, against the oracle; 100 x 75 pins the non-square path.  A data set
    without over-called SNPs still takes the triangle (k_scan_gw, LDS per wave halved)."""
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(4, [5000, 3100, 2200, 700], n1p, n2p, seed=515 + n1p)
    q = _overcall(p, n1p, n2p, 0.03, seed=n1p)
    ocfg = O.Cfg(n1p, n2p)
    bgs = O.chrom_backgrounds(q, ocfg)
    for mode, ws in ((L.WINDOW_BP, 30000), (L.WINDOW_SNPS, 120)):
        wins = O.snp_windows(q, ws)[0] if mode == L.WINDOW_SNPS else O.bp_windows(q, ws)
        _records_vs_oracle(q, ScanConfig(n1p=n1p, n2p=n2p, window_mode=mode, window=ws, fst=fst), ocfg, wins,
                           lambda c: bgs[c])
    eng = Engine.get(0)
    for data in (q, p):
        dev = eng.upload(data)
        pl = eng.plan(dev, ScanConfig(n1p=n1p, n2p=n2p, window=30000, fst=fst))
        assert pl.scan_kernel() == "k_scan_gw"
        pl.run()
        pl.check()
        if fst:
            recs, got = pl.read(), pl.read_fst()
            live = (recs["flags"][: len(got)] & L.W_EMPTY) == 0
            wins = O.bp_windows(data, 30000)
            assert int(live.sum()) == len(wins)
            for g, (c, st, b, e) in list(zip(got[live], wins))[::5]:
                assert _fst_close(float(g), O.window_fst(data, np.arange(b, e), ocfg)), (g, b, e)
        pl.close()
        dev.close()


@pytest.mark.parametrize("n1p", [50, 100])
def test_overcalled_supplied_background_sims_shape(n1p):
    """The same over-called SNPs under a supplied background (sims_scan / scan_chooseChr shape: square
    folded grid, k_scan_gw): such data sets take the bins pipeline (k_prep validates every SNP), never the
    triangle; records against the oracle with the background of the whole data set."""
    from sfs2d import _lib as L
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [4000, 2500, 900], n1p, n1p, seed=77 + n1p)
    q = _overcall(p, n1p, n1p, 0.02, seed=3 * n1p)
    ocfg = O.Cfg(n1p, n1p)
    idx = np.arange(q.n)
    bg = (O.sfs2d(q, idx, ocfg), O.fold1d(O.sfs1d(q, idx, 1, ocfg)), O.fold1d(O.sfs1d(q, idx, 2, ocfg)))
    for mode, ws in ((L.WINDOW_BP, 20000), (L.WINDOW_SNPS, 150)):
        wins = O.snp_windows(q, ws)[0] if mode == L.WINDOW_SNPS else O.bp_windows(q, ws)
        _records_vs_oracle(q, ScanConfig(n1p=n1p, n2p=n1p, window_mode=mode, window=ws, bg_mode=L.BG_SUPPLIED),
                           ocfg, wins, lambda c: bg, bg=bg)


@pytest.mark.gpu
@pytest.mark.parametrize("ws,n1p,n2p", [(100000, 11, 11), (500000, 11, 11), (500000, 18, 14), (2000000, 25, 25)])
def test_sparse_windows_all_present(ws, n1p, n2p):
    """LD-pruned real SNPs (tests/golden/vcf_test.vcf.gz via the native parser): every non-empty
    fixed-bp window is scanned with exactly its SNP range, whatever wave of its workgroup owns it
    (a grid whose replica table is smaller than the workgroup once left waves without their first
    window)."""
    import os
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.vcf import read_vcf
    g = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    p = read_vcf(os.path.join(g, "vcf_test.vcf.gz"), os.path.join(g, "popmap_3pop.txt")).to_packed("uv", "bv")
    eng = Engine.get(0)
    dev = eng.upload(p)
    try:
        recs = eng.scan(dev, ScanConfig(n1p=n1p, n2p=n2p, window=ws))
    finally:
        dev.close()
    got = {(int(r["chrom"]), int(r["wid"])): (int(r["begin"]), int(r["end"])) for r in recs
           if not r["flags"] & L.W_EMPTY}
    exp = {}
    for c in range(p.nchrom):
        lo, hi = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
        w = (p.pos[lo:hi].astype(np.int64) - 1) // ws
        for u in np.unique(w):
            ii = np.nonzero(w == u)[0]
            exp[(c, int(u))] = (lo + int(ii[0]), lo + int(ii[-1]) + 1)
    assert got == exp


def test_many_snps_in_one_bin_small_grid():
    """k_scan_w counts the 2D SFS in u16-packed bins and ranks each SNP in its bin by the atomic's return
    value (D(r) from the LDS table for r < 512, the global ln table beyond): windows of 1,000 identical
    SNPs (one bin, ranks past the LDS table) among ordinary ones, SNP-count and fixed-bp windows, against
    the oracle.  (Round 4's k_scan_wl, which wrapped u8 bins here, was removed in round 5.)"""
    from sfs2d.engine import ScanConfig
    from sfs2d.pack import PackedSNPs
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [6000, 3000], 25, 25, seed=77)
    c = p.counts.copy()
    c[1000:2000] = c[1000]          # one bin, 1,000 SNPs (SNP-count windows of 500: two wrapped windows)
    c[4000:4700] = c[4001]
    q = PackedSNPs(c, p.pos, p.chrom_off, p.chrom_names, p.ann_id, p.ann_names, p.pop1, p.pop2)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(q, ocfg)
    from sfs2d import _lib as L
    wins, _ = O.snp_windows(q, 500)
    _records_vs_oracle(q, ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=500), ocfg, wins,
                       lambda k: bgs[k])
    _records_vs_oracle(q, ScanConfig(n1p=25, n2p=25, window=200000), ocfg, O.bp_windows(q, 200000), lambda k: bgs[k])


@pytest.mark.parametrize("env", ["SFS2D_FUSED=1", "SFS2D_FUSED=0"])
def test_scan_kernels_agree(monkeypatch, env):
    """k_scan_w with its table built in the prologue (fused) and from k_bg_slice's (sliced): both against
    the oracle on fixed-bp and SNP-count windows, with Fst."""
    k, v = env.split("=")
    monkeypatch.setenv(k, v)
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(3, [9000, 4000, 1], 25, 25, seed=1234)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    _records_vs_oracle(p, ScanConfig(n1p=25, n2p=25, window=20000, fst=True), ocfg, O.bp_windows(p, 20000),
                       lambda c: bgs[c])
    wins, _ = O.snp_windows(p, 700)
    _records_vs_oracle(p, ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=700), ocfg, wins,
                       lambda c: bgs[c])
    eng = Engine.get(0)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
    pl.run()
    pl.check()
    recs, fst = pl.read(), pl.read_fst()
    live = (recs["flags"] & L.W_EMPTY) == 0
    for i in np.nonzero(live)[0][::7]:
        b, e = int(recs["begin"][i]), int(recs["end"][i])
        want = O.window_fst(p, np.arange(b, e), ocfg)
        a = float(fst[i])
        assert (np.isnan(a) if want is None else abs(a - want) <= 1e-12 + 1e-10 * abs(want)), (i, a, want)
    pl.close()
    dev.close()


@pytest.mark.parametrize("env", ["SFS2D_FUSED=1", "SFS2D_FUSED=0", "SFS2D_FST_SCAN=0"])
def test_fst_low_called_counts(monkeypatch, env):
    """SNPs with fewer than 2 called alleles in ONE population leave Hudson's Fst sums (oracle.window_fst
    keeps SNPs with >= 2 in both): the scan kernels' per-SNP terms (k_scan_w's, fused and sliced, k_prep's
    fixed-point sums) must drop them whatever the other population holds."""
    k, v = env.split("=")
    monkeypatch.setenv(k, v)
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [7000, 3000], 25, 25, seed=99)
    c = p.counts.copy()
    rng = np.random.default_rng(5)
    low = rng.choice(len(c), size=len(c) // 6, replace=False)
    pair = rng.integers(0, 3, size=len(low))                    # (ref, alt) = (0, 0), (1, 0), (0, 1)
    r, a = np.array([0, 1, 0], np.uint32)[pair], np.array([0, 0, 1], np.uint32)[pair]
    side = rng.integers(0, 2, size=len(low)).astype(bool)       # population 1 or 2
    c[low[side]] = (c[low[side]] & 0xffff0000) | r[side] | (a[side] << 8)
    c[low[~side]] = (c[low[~side]] & 0x0000ffff) | (r[~side] << 16) | (a[~side] << 24)
    p.counts = c
    ocfg = O.Cfg(25, 25)
    eng = Engine.get(0)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
    pl.run()
    pl.check()
    recs, fst = pl.read(), pl.read_fst()
    live = np.nonzero((recs["flags"][: len(fst)] & L.W_EMPTY) == 0)[0]
    assert len(live) > 20
    for i in live:
        b, e = int(recs["begin"][i]), int(recs["end"][i])
        want = O.window_fst(p, np.arange(b, e), ocfg)
        assert _fst_close(float(fst[i]), want), (i, float(fst[i]), want)
    pl.close()
    dev.close()
