"""Multi-GPU host logic on CPU: chromosome sharding, the per-rank scan ranges (with the Q9 context
chromosome), the gloo all-gather of record tables across 2 processes, and the merge into the table a
single plan over all chromosomes emits.  Per-rank records come from the oracle (tests/fake_records),
so this runs without a GPU; the GPU path uses the same functions with the RCCL backend."""
import os
import socket
import tempfile

import numpy as np
import pytest

import fake_records as FR
from oracle import sfs_oracle as O
from sfs2d import _lib as L
from sfs2d import dist as D
from sfs2d import post
from sfs2d.synth import synth_genome


def test_shard_chromosomes_balanced_and_contiguous():
    off = np.cumsum([0, 100, 5, 300, 40, 40, 200, 10])
    for world in (1, 2, 3, 4, 8, 16):
        sh = D.shard_chromosomes(off, world)
        assert len(sh) == world
        assert sh[0][0] == 0 and sh[-1][1] == len(off) - 1
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        assert all(lo <= hi for lo, hi in sh)
    sh = D.shard_chromosomes(off, 2)
    sizes = [int(off[hi] - off[lo]) for lo, hi in sh]
    assert max(sizes) <= 450   # 695 SNPs: a greedy cut near the half


def test_scan_range_adds_context_chromosome_to_last_rank():
    sh = [(0, 2), (2, 5), (5, 5)]
    assert D.scan_range(sh, 0, True) == (0, 2)
    assert D.scan_range(sh, 1, True) == (1, 5)     # last non-empty rank
    assert D.scan_range(sh, 1, False) == (2, 5)
    assert D.scan_range(sh, 2, True) == (5, 5)


def _local_tables(p, shards, ws, ocfg, bgs):
    tabs = []
    last = max(r for r, (a, b) in enumerate(shards) if b > a)
    for r in range(len(shards)):
        lo, hi = D.scan_range(shards, r, True)
        if shards[r][1] <= shards[r][0]:
            tabs.append(np.zeros(0, dtype=L.WINDOW_DTYPE))
            continue
        sub = p.subset_chroms(range(lo, hi))
        tabs.append(FR.bp_records(sub, ws, ocfg, lambda c, lo=lo: bgs[lo + c], prev_extra=(r == last)))
    return tabs


@pytest.mark.parametrize("world", [2, 3, 5])
def test_merge_equals_single_plan(world):
    p = synth_genome(4, [3000, 1500, 800, 1], 25, 25, seed=5)   # last chromosome: a single window
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    ws = 20000
    full = FR.bp_records(p, ws, ocfg, lambda c: bgs[c], prev_extra=True)
    shards = D.shard_chromosomes(p.chrom_off, world)
    merged = D.merge_tables(_local_tables(p, shards, ws, ocfg, bgs), shards, True, p.chrom_off)
    assert _same(merged, full)
    ref = O.combined_scan(p, ws, ocfg)
    got = post.combined_scan(merged, p, ws, post.num_slots(merged))
    assert list(got) == list(ref)


def _same(a, b):
    """Tables equal, except the Q9 helper's window-id field (a SNP index on the GPU, unused)."""
    a, b = a.copy(), b.copy()
    for t in (a, b):
        t["wid"][(t["flags"] & L.W_EXTRA) != 0] = 0
    return a.tobytes() == b.tobytes()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = synth_genome(3, [2500, 1200, 700], 25, 25, seed=11)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    shards = D.shard_chromosomes(p.chrom_off, world)
    local = _local_tables(p, shards, 20000, ocfg, bgs)[rank]
    tables = D.gather_tables(local, world)
    if rank == 0:
        merged = D.merge_tables(tables, shards, True, p.chrom_off)
        np.save(os.path.join(outdir, "merged.npy"), merged.view(np.uint8))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_allgather_two_ranks():
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        merged = np.load(os.path.join(d, "merged.npy")).view(L.WINDOW_DTYPE)
    p = synth_genome(3, [2500, 1200, 700], 25, 25, seed=11)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    full = FR.bp_records(p, 20000, ocfg, lambda c: bgs[c], prev_extra=True)
    assert _same(merged, full)


def run_dist_workers(mode, world, out, extra=(), timeout=600, env_extra=None):
    """Start `world` rank processes of tests/dist_worker.py (gloo on 127.0.0.1); returns rank 0's
    JSON (every golden driver call, scanned sharded)."""
    import json
    import subprocess
    import sys
    port = _free_port()
    here = os.path.dirname(os.path.abspath(__file__))
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   OMP_NUM_THREADS="1", **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(here, "dist_worker.py"), mode, out, *extra],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for q in procs:
            o, _ = q.communicate(timeout=timeout)
            logs.append(o.decode(errors="replace"))
    finally:
        for q in procs:
            if q.poll() is None:
                q.kill()
    assert all(q.returncode == 0 for q in procs), "\n".join(x[-3000:] for x in logs)
    with open(out) as fh:
        return json.load(fh)


def check_dist_results(got, golden):
    """Every call's sharded result equals the reference's (golden) result or error."""
    import golden_util as gu
    n = 0
    for name in golden.cases():
        for i, c in enumerate(golden.calls(name)):
            key = f"{name}-{i}"
            if key not in got:
                continue
            n += 1
            g, ref = got[key], c["out"]
            if c["fn"] == "sims_process_window":
                assert g["ok"], (key, g)
                errs = gu.compare_results(gu.decode_results(g["results"]), gu.decode_results(ref["results"]))
                assert not errs, (key, errs[:5])
                continue
            if not ref["ok"]:
                assert not g["ok"] and g["error"] == ref["error"], (key, g)
                continue
            assert g["ok"], (key, g)
            errs = gu.compare_results(gu.decode_results(g["results"]), gu.decode_results(ref["results"]))
            assert not errs, (key, errs[:5])
    return n


@pytest.mark.parametrize("world,mode", [(2, "split"), (3, "split"), (2, "chromosomes")])
def test_sharded_drivers_vs_reference(golden, tmp_path, world, mode):
    """Every golden driver call (combined_scan, scan_chooseChr, scan_precomputed_BG, both bySNPs
    drivers, T1D_scan / T2D_scan, the sims batch) through the drop-in modules with distributed=True
    over `world` gloo ranks: split at window boundaries (chromosomes cut across ranks, background
    histograms all-reduced) or sharded by whole chromosomes, per-rank scan (the oracle's records in
    place of the GPU's), collective error handling, gather, merge, post-pass -- equal to the
    reference's outputs."""
    env = {"SFS2D_TEST_DIST": "chromosomes"} if mode == "chromosomes" else None
    got = run_dist_workers("fake", world, str(tmp_path / "out.json"), env_extra=env)
    assert check_dist_results(got, golden) >= 40
    st = got["_stats"]
    if mode == "split":
        # most calls ran split (the error cases fall back to whole chromosomes), with all-reduces
        assert st["split"] >= 30 and st["allreduce"] >= 10, st
        assert st["fallback"] <= 12, st


def test_split_error_falls_back_to_whole_chromosomes(tmp_path):
    """A count error in each rank's part of one chromosome: the error the reference raises (its
    whole-chromosome 2D background comes first: ValueError) on every rank, via the fallback."""
    got = run_dist_workers("fake", 2, str(tmp_path / "out.json"), extra=("errors",))
    for fn in ("combined_scan", "scan_perChr_bySNPs"):
        assert got[fn]["ref"] == "ValueError"
        assert not got[fn]["ok"] and got[fn]["error"] == "ValueError", got[fn]
    assert got["_stats"]["fallback"] == 2, got["_stats"]


@pytest.mark.parametrize("world", [2, 3])
def test_single_chromosome_split_equals_one_rank_cpu(tmp_path, world):
    got = run_dist_workers("fake", world, str(tmp_path / "out.json"), extra=("single",))
    check_single(got)


def check_single(got):
    for name in ("bp_perchrom", "bp_perchrom_nofold_filters", "snp_perchrom", "bp_supplied"):
        assert got[name]["equal"] and got[name]["windows"] > 50, (name, got[name])
    assert got["_stats"]["split"] == 4 and got["_stats"]["allreduce"] == 3 and got["_stats"]["fallback"] == 0


def test_split_points_whole_windows_balanced():
    from sfs2d.engine import ScanConfig
    p = synth_genome(3, [4000, 300, 2500], 25, 25, seed=21)
    for mode, w in ((L.WINDOW_BP, 20000), (L.WINDOW_SNPS, 300)):
        for pe in (False, True):
            cfg = ScanConfig(n1p=25, n2p=25, window_mode=mode, window=w, prev_extra=pe)
            starts = set(D.window_starts(p, cfg).tolist())
            for world in (1, 2, 3, 4, 7, 64):
                cuts = D.split_points(p, cfg, world)
                assert cuts[0] == 0 and cuts[-1] == p.n and len(cuts) == world + 1
                assert all(a <= b for a, b in zip(cuts, cuts[1:]))
                assert all(c in starts for c in cuts[1:-1] if c < p.n)
                if world <= 4:
                    assert max(b - a for a, b in zip(cuts, cuts[1:])) <= p.n / world + 2 * (w if mode == L.WINDOW_SNPS else 400)
                if pe:   # the last non-empty rank holds the last two windows
                    last = max(r for r in range(world) if cuts[r + 1] > cuts[r])
                    assert cuts[last] <= sorted(starts)[-2]


def test_split_merge_equals_single_plan():
    """Per-part tables (oracle records over each rank's SNP range, backgrounds of the whole
    chromosomes) merged = one plan's table minus its empty slots."""
    from sfs2d.engine import ScanConfig
    p = synth_genome(2, [3000, 2000], 25, 25, seed=8)
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(p, ocfg)
    for world in (2, 3, 5):
        cfg = ScanConfig(n1p=25, n2p=25, window=20000, prev_extra=True)
        cuts = D.split_points(p, cfg, world)
        last = max(r for r in range(world) if cuts[r + 1] > cuts[r])
        tabs, c0s = [], []
        for r in range(world):
            sub, c0 = p.slice_snps(cuts[r], cuts[r + 1])
            c0s.append(c0)
            tabs.append(FR.bp_records(sub, 20000, ocfg, lambda c, c0=c0: bgs[c0 + c], prev_extra=(r == last))
                        if sub.n else np.zeros(0, dtype=L.WINDOW_DTYPE))
        merged = D._merge_split(tabs, cuts, c0s, True)
        full = FR.bp_records(p, 20000, ocfg, lambda c: bgs[c], prev_extra=True)
        full = full[((full["flags"] & L.W_EMPTY) == 0) | ((full["flags"] & L.W_EXTRA) != 0)]
        assert _same(merged, full), world
        assert list(post.combined_scan(merged, p, 20000, post.num_slots(merged))) == list(O.combined_scan(p, 20000, ocfg))
