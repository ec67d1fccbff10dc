"""The native multi-GPU step loop (sfs2d_dist_*, include/sfs2d.h): RCCL loaded at run time, one
communicator per rank, scans and all-gathers of the window tables enqueued from C.  On the one-GPU
box: a one-rank communicator (gather and all-gather are copies) -- the tables gathered after back-to-back
steps equal the plan's own records.  N > 1 runs are the driver's (bench.py --gpus N)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_single_rank_scan_gather():
    import torch
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [30000, 9000], 25, 25, seed=21)
    eng = Engine.get(0)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=25, n2p=25, window=20000, fst=True))
    pl.run()
    pl.check()
    ref = pl.read()
    rows = pl.nrec + 3   # padded like bench.py's shards
    outs = [torch.zeros((rows, 64), dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    gath = [torch.full((rows, 64), 7, dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    comm = torch.cuda.Stream(device=0)
    d = eng.dist(eng.dist_unique_id(), 0, 1)
    try:
        # overlapped gathers to the root, serial gathers to the root, serial all-gathers
        for first, n, cs, root in ((0, 5, comm.cuda_stream, True), (5, 4, None, True), (9, 3, None, False)):
            d.set_gather(root)
            for g in gath:
                g.fill_(7)
            d.scan_gather(pl, [o.data_ptr() for o in outs], [g.data_ptr() for g in gath], rows, first, n, cs)
            torch.cuda.synchronize()
            pl.check()
            for o, g in zip(outs, gath):
                assert torch.equal(o, g)
                recs = np.frombuffer(o[: pl.nrec].cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
                assert recs.tobytes() == ref.tobytes()
        with pytest.raises(L.Sfs2dError):   # rows must cover the plan's records
            d.scan_gather(pl, [o.data_ptr() for o in outs], [g.data_ptr() for g in gath], pl.nrec - 1, 0, 1,
                          comm.cuda_stream)
    finally:
        d.close()
        pl.close()


def test_single_rank_scan_gather_streams():
    """sfs2d_dist_scan_gather_streams: steps in groups over two plans on two streams, one gather of a
    group's tables per group (to the root and all-gathered), a last partial group; every table and
    every gathered copy equals the plan's own records; argument errors."""
    import torch
    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(2, [30000, 9000], 25, 25, seed=22)
    eng = Engine.get(0)
    dev = eng.upload(p)
    cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=True)
    plans = [eng.plan(dev, cfg) for _ in range(2)]
    plans[0].run()
    plans[0].check()
    ref = plans[0].read()
    rows = plans[0].nrec + 2
    outbuf = torch.zeros((4 * rows, 64), dtype=torch.uint8, device="cuda:0")
    gath = [torch.full((2 * rows, 64), 7, dtype=torch.uint8, device="cuda:0") for _ in range(2)]
    streams = [torch.cuda.Stream(device=0).cuda_stream for _ in range(2)]
    d = eng.dist(eng.dist_unique_id(), 0, 1)
    gp = [g.data_ptr() for g in gath]
    try:
        for root, nsteps in ((True, 8), (False, 8), (True, 5)):
            d.set_gather(root)
            outbuf.zero_()
            for g in gath:
                g.fill_(7)
            d.scan_gather_streams(plans, streams, outbuf.data_ptr(), gp, rows, nsteps)
            torch.cuda.synchronize()
            for q in plans:
                q.check()
            tabs = outbuf.view(4, rows, 64)
            # 5 steps: groups (0, 1), (2, 3), (4): tables 0-3 written, group 2 (parity 0) gathers table 0 only
            for t in range(4):
                recs = np.frombuffer(tabs[t][: rows - 2].cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
                assert recs.tobytes() == ref.tobytes(), (root, nsteps, t)
            for par in range(2):
                assert torch.equal(gath[par][: rows - 2], tabs[2 * par][: rows - 2])
                if nsteps == 8:
                    assert torch.equal(gath[par], outbuf[2 * par * rows: (2 * par + 2) * rows])
        with pytest.raises(L.Sfs2dError):   # one plan twice
            d.scan_gather_streams([plans[0], plans[0]], streams, outbuf.data_ptr(), gp, rows, 2)
        with pytest.raises(L.Sfs2dError):   # rows must cover the records
            d.scan_gather_streams(plans, streams, outbuf.data_ptr(), gp, rows - 3, 2)
    finally:
        d.close()
        for q in plans:
            q.close()
