"""The C ABI's stream contract (include/sfs2d.h, sfs2d_ctx_set_stream / sfs2d_ctx_use_own_stream): a scan
enqueued on a stream shared with torch runs after the torch work queued before it on that stream -- the
default stream (handle 0, the HIP null stream) included.  Round 4 found a NaN background when handle 0
silently selected the library's own unordered stream (sfs2d/dist.py _one_stream); this pins the order
deterministically: the scan's inputs are written by torch behind ~20 ms of queued matmuls, so an
unordered scan would read the zero-filled buffers.  (The reference object is single-threaded and
stateful, twoDSFS_class.py:21-33; the ctx + stream is the state it becomes here.)"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
@pytest.mark.parametrize("which", ["default", "side"])
def test_scan_ordered_after_torch_fill_on_shared_stream(which):
    import torch
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(4, 1_000_000, 25, 25, seed=8)
    cfg = ScanConfig(n1p=25, n2p=25, window=20000, fst=True)
    eng = Engine.get(0)
    ref = eng.upload(p)
    want = eng.scan(ref, cfg)
    ref.close()
    dev = torch.device("cuda:0")
    counts = torch.zeros(p.n + 64, dtype=torch.int32, device=dev)
    pos = torch.zeros(p.n + 64, dtype=torch.int32, device=dev)
    src_c = torch.from_numpy(p.counts.view(np.int32)).to(dev)
    src_p = torch.from_numpy(p.pos.view(np.int32)).to(dev)
    last_pos = p.pos[p.chrom_off[1:] - 1]
    torch.cuda.synchronize()
    s = torch.cuda.default_stream(dev) if which == "default" else torch.cuda.Stream(device=dev)
    if which == "default":
        assert s.cuda_stream == 0   # torch's default stream is the HIP null stream
    prev = eng.set_stream(s.cuda_stream)
    try:
        d = eng.wrap_device(counts.data_ptr(), pos.data_ptr(), None, p.n, p.chrom_off, last_pos)
        pl = eng.plan(d, cfg)
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            x = torch.randn(4096, 4096, device=dev)
            for _ in range(16):   # ~20 ms queued ahead of the fill
                x = x @ x
                x = x / x.norm()
            counts[:p.n].copy_(src_c)
            pos[:p.n].copy_(src_p)
            pl.run()              # enqueued on s, behind the fill
        got = pl.read()           # (synchronises s)
        pl.check()
        pl.close()
        d.close()
    finally:
        eng.set_stream(prev)
    assert len(got) == len(want)
    assert got.tobytes() == want.tobytes()
