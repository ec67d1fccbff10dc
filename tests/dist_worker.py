"""Test-only: one rank of a sharded run of every golden driver call (tests/golden/manifest.json)
through the drop-in modules with ``distributed=True`` (sfs2d.dist.scan_records).

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


def fake_scan(sub, cfg, bg):
    """What Engine.scan returns for ``sub`` / ScanConfig ``cfg``, built by the oracle."""
    import fake_records as FR
    from sfs2d import _lib as L
    vt = None
    if cfg.ann_want >= 0:
        vt = sub.ann_names[cfg.ann_want] if cfg.ann_want < len(sub.ann_names) else "\x00absent"
    ocfg = O.Cfg(cfg.n1p, cfg.n2p, vt, cfg.fold, cfg.start_position, cfg.end_position)
    if cfg.bg_mode == L.BG_PER_CHROM:
        bgs = O.chrom_backgrounds(sub, ocfg)
        bg_of = lambda c: bgs[c]
    else:
        b = (np.asarray(bg[0], np.float64).reshape(-1), np.asarray(bg[1], np.float64), np.asarray(bg[2], np.float64))
        if all(float(x) == int(x) for x in np.concatenate(b)):   # integer backgrounds: exact ints, as the kernel
            b = tuple(x.astype(np.int64) for x in b)
        bg_of = lambda c: b
    if cfg.window_mode == L.WINDOW_BP:
        return FR.bp_records(sub, cfg.window, ocfg, bg_of, prev_extra=cfg.prev_extra)
    return FR.snp_records(sub, cfg.window, ocfg, bg_of)


def _class_obj(cfgd, mode):
    import twoDSFS_class as T
    obj = T.LikelihoodInference_jointSFS(None, None, start_position=cfgd.get("start_position"),
                                         end_position=cfgd.get("end_position"), pop1=cfgd["pop1"],
                                         pop2=cfgd["pop2"], pop1_size=cfgd["n1p"], pop2_size=cfgd["n2p"],
                                         variant_type=cfgd.get("variant_type"), fold=cfgd.get("fold", True),
                                         device=int(os.environ.get("SFS2D_DEVICE", "0")), distributed=True)
    if mode == "fake":
        obj._scan_local = fake_scan

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
                ok, res, _ = gu.run_capture(lambda: S.process_windows_batch(
                    [p, p], bg2, dict(enumerate(b1.tolist())), dict(enumerate(b1b.tolist())), 500000, "p1", "p2",
                    n, n, distributed=True)[1])
            else:
                obj = _class_obj(cfgd, mode)
                ok, res, _ = gu.run_capture(call, obj, p, cfgd, c["fn"], c["args"])
            out[f"{name}-{i}"] = ({"ok": True, "results": gu.enc_results(res)} if ok else
                                  {"ok": False, "error": type(res).__name__, "message": str(res)})
    if dist.get_rank() == 0:
        with open(out_path, "w") as fh:
            json.dump(out, fh)
    dist.barrier()


def main():
    import torch.distributed as dist
    mode, out_path = sys.argv[1], sys.argv[2]
    dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
    try:
        run_all(mode, out_path, skip=() if len(sys.argv) > 3 and sys.argv[3] == "all" else ("chr1",))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
