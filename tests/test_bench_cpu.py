"""bench.py's host logic on CPU: the headline's shards (config 3 split by window over N ranks) and the
window count of a gathered table, with a gloo world-2 all-gather of per-rank record tables built by
the oracle (the GPU loop around them is the same at every N)."""
import os
import socket
import sys
import tempfile

import numpy as np
import pytest

import fake_records as FR
from oracle import sfs_oracle as O
from sfs2d import _lib as L
from sfs2d.engine import ScanConfig
from sfs2d.synth import synth_genome

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _genome():
    # config 3's shape, scaled down: 8 equal chromosomes
    return synth_genome(8, 6000, 25, 25, seed=9)


@pytest.mark.parametrize("world", [1, 2, 4, 8, 3])
def test_config3_cuts(world):
    p = _genome()
    cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=True, scan_wgs_per_cu=1)
    cuts = bench.config3_cuts(p, cfg, world)
    assert cuts[0] == 0 and cuts[-1] == p.n and len(cuts) == world + 1
    assert all(a <= b for a, b in zip(cuts, cuts[1:]))
    ends = set(p.chrom_off.tolist())
    assert all(c in ends for c in cuts)   # whole chromosomes: no background exchange in the timed loop
    if 8 % world == 0:   # N | nchrom: equal shards
        sizes = np.diff(cuts)
        assert sizes.min() == sizes.max() == p.n // world


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = _genome()
    cfg = ScanConfig(n1p=25, n2p=25, window=20000)
    cuts = bench.config3_cuts(p, cfg, world)
    sub, _ = p.slice_snps(cuts[rank], cuts[rank + 1])
    ocfg = O.Cfg(25, 25)
    bgs = O.chrom_backgrounds(sub, ocfg)
    mine = FR.bp_records(sub, 20000, ocfg, lambda c: bgs[c]).view(np.uint8).reshape(-1, 64)
    n = torch.tensor([len(mine)])
    dist.all_reduce(n, op=dist.ReduceOp.MAX)
    rows = int(n.item())
    out = torch.zeros((rows, 64), dtype=torch.uint8)
    out[len(mine):, 39] = 0x80   # padding rows flagged empty, as bench.run_loop pads its tables
    out[: len(mine)] = torch.from_numpy(mine.copy())
    g = torch.empty((world * rows, 64), dtype=torch.uint8)
    dist.all_gather_into_tensor(g, out)
    if rank == 0:
        np.save(os.path.join(outdir, "n.npy"), np.array([bench.n_windows(g.numpy())]))
    dist.barrier()
    dist.destroy_process_group()


def test_gathered_window_count_world2():
    import torch.multiprocessing as mp
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        got = int(np.load(os.path.join(d, "n.npy"))[0])
    p = _genome()
    want = len(O.bp_windows(p, 20000))
    assert got == want
