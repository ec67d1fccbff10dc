"""Test-only: one rank of a sharded run of every golden driver call (tests/golden/manifest.json)
through the drop-in modules with ``distributed=True`` (split at window boundaries,
sfs2d.dist.scan_records_split; SFS2D_TEST_DIST=chromosomes: whole-chromosome shards,
sfs2d.dist.scan_records).

mode "gpu": each rank scans its chromosome shard with the HIP library on GPU ``SFS2D_DEVICE``
(several ranks may share one GPU); mode "fake": the per-rank scan is the oracle's record builder
(tests/fake_records.py), so the sharding / gather / merge / post-pass logic runs on CPU.  The group
is gloo (tables exchanged on the host).  Rank 0 writes {case-i: {"ok", "results" | "error"}} as JSON.

    RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python tests/dist_worker.py gpu out.json
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for q in (os.path.join(REPO, "2dsfs-scan_amd"), REPO, HERE):
    if q not in sys.path:
        sys.path.insert(0, q)

import numpy as np  # noqa: E402

import golden_util as gu  # noqa: E402
from oracle import sfs_oracle as O  # noqa: E402


def _ocfg(cfgd):
    return O.Cfg(cfgd["n1p"], cfgd["n2p"], cfgd.get("variant_type"), cfgd.get("fold", True),
                 cfgd.get("start_position"), cfgd.get("end_position"))


def _fake_ocfg(sub, cfg):
    vt = None
    if cfg.ann_want >= 0:
        vt = sub.ann_names[cfg.ann_want] if cfg.ann_want < len(sub.ann_names) else "\x00absent"
    return O.Cfg(cfg.n1p, cfg.n2p, vt, cfg.fold, cfg.start_position, cfg.end_position)


def _fake_records(sub, cfg, ocfg, bg_of):
    import fake_records as FR
    from sfs2d import _lib as L
    if cfg.window_mode == L.WINDOW_BP:
        return FR.bp_records(sub, cfg.window, ocfg, bg_of, prev_extra=cfg.prev_extra)
    return FR.snp_records(sub, cfg.window, ocfg, bg_of)


def _supplied(bg):
    b = (np.asarray(bg[0], np.float64).reshape(-1), np.asarray(bg[1], np.float64), np.asarray(bg[2], np.float64))
    if all(float(x) == int(x) for x in np.concatenate(b)):   # integer backgrounds: exact ints, as the kernel
        b = tuple(x.astype(np.int64) for x in b)
    return b


def fake_scan(sub, cfg, bg):
    """What Engine.scan returns for ``sub`` / ScanConfig ``cfg``, built by the oracle."""
    from sfs2d import _lib as L
    ocfg = _fake_ocfg(sub, cfg)
    if cfg.bg_mode == L.BG_PER_CHROM:
        bgs = O.chrom_backgrounds(sub, ocfg)
        bg_of = lambda c: bgs[c]
    else:
        b = _supplied(bg)
        bg_of = lambda c: b
    return _fake_records(sub, cfg, ocfg, bg_of)


class FakeSplitJob:
    """sfs2d.engine.SplitJob with the oracle in place of the GPU: partial() = the part's unfolded
    2D / 1D histograms per chromosome, finish(total) = records against the summed histograms."""

    def __init__(self, sub, cfg, bg):
        self.sub, self.cfg, self.bg = sub, cfg, bg
        self.ocfg = _fake_ocfg(sub, cfg)

    def partial(self):
        from sfs2d import _lib as L
        if self.cfg.bg_mode != L.BG_PER_CHROM:
            return None
        rows = []
        for c in range(self.sub.nchrom):   # the exchange's row layout (sfs2d.dist.hist_width)
            idx = np.arange(self.sub.chrom_off[c], self.sub.chrom_off[c + 1])
            h2 = O.sfs2d(self.sub, idx, self.ocfg).ravel()
            rows.append(np.concatenate([h2, O.sfs1d(self.sub, idx, 1, self.ocfg), O.sfs1d(self.sub, idx, 2, self.ocfg),
                                        [h2[1:-1].sum()]]))
        return np.array(rows, dtype=np.int64).reshape(self.sub.nchrom, -1)

    def finish(self, total):
        if total is None:
            b = _supplied(self.bg)
            return _fake_records(self.sub, self.cfg, self.ocfg, lambda c: b)
        n1, n2 = 2 * self.cfg.n1p, 2 * self.cfg.n2p
        nb = (n1 + 1) * (n2 + 1)
        bgs = [(t[:nb].reshape(n1 + 1, n2 + 1), O.fold1d(t[nb:nb + n1 + 1]), O.fold1d(t[nb + n1 + 1:nb + n1 + n2 + 2]))
               for t in np.asarray(total, np.int64)]
        return _fake_records(self.sub, self.cfg, self.ocfg, lambda c: bgs[c])

    def close(self):
        pass


def _class_obj(cfgd, mode):
    import twoDSFS_class as T
    obj = T.LikelihoodInference_jointSFS(None, None, start_position=cfgd.get("start_position"),
                                         end_position=cfgd.get("end_position"), pop1=cfgd["pop1"],
                                         pop2=cfgd["pop2"], pop1_size=cfgd["n1p"], pop2_size=cfgd["n2p"],
                                         variant_type=cfgd.get("variant_type"), fold=cfgd.get("fold", True),
                                         device=int(os.environ.get("SFS2D_DEVICE", "0")),
                                         distributed=os.environ.get("SFS2D_TEST_DIST", True))
    if mode == "fake":
        obj._scan_local = fake_scan
        obj._split_scan = FakeSplitJob

        def bg_arrays(p, chrom, obj=obj):
            oc = _ocfg(cfgd)
            idx = np.arange(p.chrom_off[chrom], p.chrom_off[chrom + 1])
            return O.sfs2d(p, idx, oc), O.fold1d(O.sfs1d(p, idx, 1, oc)), O.fold1d(O.sfs1d(p, idx, 2, oc))
        obj._bg_arrays = bg_arrays
    return obj


def call(obj, p, cfgd, fn, args):
    if fn == "scan_precomputed_BG":
        g2, g1a, g1b = O.genome_backgrounds_normalized(p, _ocfg(cfgd))
        n2 = 2 * cfgd["n2p"] + 1
        bg2 = {(k // n2, k % n2): float(v) for k, v in enumerate(g2.ravel())}
        return obj.scan_precomputed_BG(p, args[0], bg2, dict(enumerate(g1a.tolist())), dict(enumerate(g1b.tolist())))
    if fn in ("T2D_scan", "T1D_scan"):
        data, bg, extra = gu.t12_inputs(p, cfgd, fn, args)
        return getattr(obj, fn)(data, bg, *extra)
    return getattr(obj, fn)(p, *args)


def run_all(mode, out_path, skip=("chr1",)):
    import torch.distributed as dist
    g = gu.Golden()
    out = {}
    for name in g.cases():
        if name in skip:
            continue
        p = g.packed(name)
        cfgd = g.cfg(name)
        for i, c in enumerate(g.calls(name)):
            if c["fn"] == "sims_process_window":
                import sims_scan as S
                bgd = g.packed(f"{name}_bgdata")
                n = cfgd["n1p"]
                b2, b1, b1b = O.sims_backgrounds(bgd, n, n)
                bg2 = {(a, b): int(b2[a, b]) for a in range(2 * n + 1) for b in range(2 * n + 1)}
                if mode == "fake":
                    S._scan_local = fake_scan
                    S._split_scan = FakeSplitJob
                ok, res, _ = gu.run_capture(lambda: S.process_windows_batch(
                    [p, p], bg2, dict(enumerate(b1.tolist())), dict(enumerate(b1b.tolist())), 500000, "p1", "p2",
                    n, n, distributed=True)[1])
            else:
                obj = _class_obj(cfgd, mode)
                ok, res, _ = gu.run_capture(call, obj, p, cfgd, c["fn"], c["args"])
            out[f"{name}-{i}"] = ({"ok": True, "results": gu.enc_results(res)} if ok else
                                  {"ok": False, "error": type(res).__name__, "message": str(res)})
    from sfs2d import dist as D
    out["_stats"] = dict(D.STATS)
    if dist.get_rank() == 0:
        with open(out_path, "w") as fh:
            json.dump(out, fh)
    dist.barrier()


def run_errors(mode, out_path):
    """One chromosome whose halves hold different bad SNPs: a 1D-only count error (alt1 above
    2 * pop1_size, folded out of the 2D grid: KeyError) in rank 0's part, a 2D grid error
    (ValueError) in rank 1's.  The reference computes the whole chromosome's 2D background first, so
    it raises ValueError; the split scan must fall back to whole chromosomes to raise the same."""
    import torch.distributed as dist
    from sfs2d import dist as D
    from sfs2d.pack import pack_counts
    from sfs2d.synth import synth_genome
    p = synth_genome(1, [4000], 25, 25, seed=3)
    r1, a1, r2, a2 = p.ref1, p.alt1, p.ref2, p.alt2
    r1[500], a1[500], r2[500], a2[500] = 0, 60, 0, 50
    r1[3500], a1[3500], r2[3500], a2[3500] = 60, 60, 0, 0
    p.counts = pack_counts(r1, a1, r2, a2)
    cfgd = {"n1p": 25, "n2p": 25, "pop1": p.pop1, "pop2": p.pop2}
    obj = _class_obj(cfgd, mode)
    out = {}
    for fn, args in (("combined_scan", [20000]), ("scan_perChr_bySNPs", [200])):
        ok, res, _ = gu.run_capture(lambda: getattr(obj, fn)(p, *args))
        out[fn] = {"ok": ok, "error": type(res).__name__, "message": str(res)} if not ok else {"ok": True}
        try:
            getattr(O, fn)(p, args[0], _ocfg(cfgd))
            out[fn]["ref"] = None
        except Exception as e:  # noqa: BLE001
            out[fn]["ref"] = type(e).__name__
    out["_stats"] = dict(D.STATS)
    if dist.get_rank() == 0:
        with open(out_path, "w") as fh:
            json.dump(out, fh)
    dist.barrier()


def run_single(mode, out_path):
    """One chromosome (config-1-like, 60k SNPs) split over the ranks: the merged record table of every
    scan kind equals, byte for byte, the table one rank's plan over the whole chromosome emits (minus
    its empty slots): per-chromosome backgrounds all-reduced (bp windows with the Q9 helper, SNP-count
    windows), and a supplied background."""
    import torch.distributed as dist
    from sfs2d import _lib as L
    from sfs2d import dist as D
    from sfs2d.engine import Engine, ScanConfig, SplitJob
    from sfs2d.synth import synth_genome
    dev = int(os.environ.get("SFS2D_DEVICE", "0"))
    p = synth_genome(1, [60000], 25, 25, seed=17)
    if mode == "gpu":
        factory = lambda sub, cfg, bg: SplitJob(Engine.get(dev), sub, cfg, bg)
        factory.device_rows = True   # background rows exchanged in HBM (sfs2d.dist._split_device)
    else:
        factory = FakeSplitJob
    bg = (np.arange(51 * 51, dtype=np.float64).reshape(51, 51) % 7 + 1, np.arange(26.0) + 1, np.arange(26.0) % 5 + 1)
    cfgs = {"bp_perchrom": ScanConfig(n1p=25, n2p=25, window=20000, prev_extra=True),
            "bp_perchrom_nofold_filters": ScanConfig(n1p=25, n2p=25, fold=False, window=7000, start_position=10 ** 5,
                                                     end_position=4 * 10 ** 6),
            "snp_perchrom": ScanConfig(n1p=25, n2p=25, window_mode=L.WINDOW_SNPS, window=500),
            "bp_supplied": ScanConfig(n1p=25, n2p=25, window=20000, bg_mode=L.BG_SUPPLIED)}
    out = {}
    for name, cfg in cfgs.items():
        b = bg if cfg.bg_mode == L.BG_SUPPLIED else None
        got = D.scan_records_split(p, cfg, b, factory, dev)
        full = D.whole_scan(factory)(p, cfg, b)
        full = full[((full["flags"] & L.W_EMPTY) == 0) | ((full["flags"] & L.W_EXTRA) != 0)]
        for t in (got, full):   # the Q9 helper's wid is its first SNP's index in the scanned data: unused
            t["wid"][(t["flags"] & L.W_EXTRA) != 0] = 0
        out[name] = {"equal": got.tobytes() == full.tobytes(), "n": int(len(full)),
                     "windows": int(((full["flags"] & L.W_EMPTY) == 0).sum())}
    out["_stats"] = dict(D.STATS)
    if dist.get_rank() == 0:
        with open(out_path, "w") as fh:
            json.dump(out, fh)
    dist.barrier()


def _strip(t):
    """A table as one plan over all SNPs leaves it for the post-pass: empty bp slots dropped, the Q9
    helper's wid (its first SNP's index in the scanned data, unused) zeroed."""
    from sfs2d import _lib as L
    t = t[((t["flags"] & L.W_EMPTY) == 0) | ((t["flags"] & L.W_EXTRA) != 0)].copy()
    t["wid"][(t["flags"] & L.W_EXTRA) != 0] = 0
    return t


def run_config3(mode, out_path, data_path):
    """BASELINE config 3 at full size (5e7 SNPs, 32 chromosomes; the parent generated it into
    ``data_path``) split over the ranks at window boundaries -- with 3 ranks the cuts fall inside
    chromosomes, so their background rows are all-reduced -- at 20 kb and 500 kb with per-chromosome
    backgrounds, and at 20 kb against the genome-wide background (the reference script's
    calculate_2d_sfs(all) -> normalize -> scan_precomputed_BG, twoDSFS_class.py:1970-1983, 1161),
    histogrammed sharded (sfs2d.dist.sharded_bg_hist).  Rank 0 compares every merged table with the
    table one GPU's plan over the whole genome writes, byte for byte."""
    import torch.distributed as dist
    from sfs2d import _lib as L
    from sfs2d import dist as D
    from sfs2d.engine import Engine, ScanConfig, SplitJob
    from sfs2d.pack import PackedSNPs
    dev = int(os.environ.get("SFS2D_DEVICE", "0"))
    z = np.load(data_path)
    p = PackedSNPs(z["counts"], z["pos"], z["chrom_off"], [f"chr{c:02d}" for c in range(len(z["chrom_off"]) - 1)],
                   None, [], "p1", "p2")
    factory = lambda sub, cfg, bg: SplitJob(Engine.get(dev), sub, cfg, bg)
    factory.device_rows = True
    rank = dist.get_rank()
    out = {}
    cfgs = {"bp20k_perchrom": (ScanConfig(n1p=25, n2p=25, window=20000, prev_extra=True), None),
            "bp500k_perchrom": (ScanConfig(n1p=25, n2p=25, window=500000, prev_extra=True), None)}
    # the genome-wide background, sharded, against one GPU's histogram of all SNPs
    hcfg = ScanConfig(n1p=25, n2p=25)
    h2, u1, u2 = D.sharded_bg_hist(p, hcfg, dev)
    if rank == 0:
        eng = Engine.get(dev)
        d = eng.upload(p)
        r2, r1, r1b = eng.bg_hist(d, hcfg, -1)
        d.close()
        out["genome_hist_equal"] = bool(np.array_equal(h2, r2) and np.array_equal(u1, r1) and np.array_equal(u2, r1b))
    # normalised as normalize_2d_sfs / normalize_1d_sfs do (sum of values[1:-1] in insertion order)
    fold = lambda u: np.bincount(np.minimum(np.arange(len(u)), len(u) - 1 - np.arange(len(u))), weights=u)
    def norm(v):
        t = sum(v[1:-1].tolist())
        return np.array([x / t for x in v.tolist()])
    bg = (norm(h2.ravel().astype(np.float64)).reshape(h2.shape), norm(fold(u1.astype(np.float64))),
          norm(fold(u2.astype(np.float64))))
    cfgs["bp20k_genome_bg"] = (ScanConfig(n1p=25, n2p=25, window=20000, bg_mode=L.BG_SUPPLIED), bg)
    for name, (cfg, b) in cfgs.items():
        before = dict(D.STATS)
        got = D.scan_records_split(p, cfg, b, factory, dev)
        split = D.STATS["split"] - before["split"]
        if rank == 0:
            full = _strip(D.whole_scan(factory)(p, cfg, b))
            got = _strip(got)
            out[name] = {"equal": got.tobytes() == full.tobytes(), "n": int(len(full)), "split": split,
                         "windows": int(((full["flags"] & L.W_EMPTY) == 0).sum())}
    out["_stats"] = dict(D.STATS)
    out["cuts"] = D.split_points(p, cfgs["bp20k_perchrom"][0], dist.get_world_size())
    if rank == 0:
        with open(out_path, "w") as fh:
            json.dump(out, fh)
    dist.barrier()


def main():
    import torch.distributed as dist
    mode, out_path = sys.argv[1], sys.argv[2]
    backend = os.environ.get("SFS2D_TEST_BACKEND", "gloo")
    if backend == "nccl":   # RCCL: the device-resident collectives of the split path (one GPU: world 1)
        import torch
        torch.cuda.set_device(int(os.environ.get("SFS2D_DEVICE", "0")))
    dist.init_process_group(backend, rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
    try:
        what = sys.argv[3] if len(sys.argv) > 3 else ""
        if what == "errors":
            run_errors(mode, out_path)
        elif what == "single":
            run_single(mode, out_path)
        elif what == "config3":
            run_config3(mode, out_path, sys.argv[4])
        else:
            run_all(mode, out_path, skip=() if what == "all" else ("chr1",))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
