"""Multi-GPU scan: chromosome shards, one process per GPU, one gather of the window tables.

Given per-chromosome backgrounds (combined_scan, scan_perChr_bySNPs; twoDSFS_class.py:809-825,
1422-1541) or one supplied background (scan_chooseChr, scan_precomputed_BG, the bySNPs driver
with a chosen chromosome, T1D_scan / T2D_scan, the sims replicates) every chromosome is
independent, so a rank scans a contiguous range of whole chromosomes with no collective on the
data path.  The only exchange is one all-gather of the fixed-stride 64-B window records
(RCCL over xGMI with the "nccl" backend on MI355X, gloo on CPU), after which the tables are
concatenated in chromosome order -- the table one plan over all chromosomes would emit -- and the
sequential rules of the drivers (sfs2d.post: stale carry Q6, final block Q9) run on it, on every
rank (``scan_records``; the drop-in class with ``distributed=True``).

The final-block helper record (Q9) needs the window before the last one of the whole scan, which
may sit in the previous chromosome: the last rank therefore also scans the chromosome before its
range (its records are dropped in the merge, the owner's are kept) and contributes the only
helper record.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L

# scan_records_split calls of this process: "split" (scans done split), "allreduce" (background
# all-reduces), "fallback" (scans redone by whole chromosomes after an error)
STATS = {"split": 0, "allreduce": 0, "fallback": 0}


def shard_chromosomes(chrom_off: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Contiguous chromosome ranges [lo, hi) per rank, balanced by SNP count (greedy cuts at
    k * total / world).  Ranks may get an empty range when there are fewer chromosomes than ranks."""
    off = np.asarray(chrom_off, dtype=np.int64)
    nchrom = len(off) - 1
    if world < 1:
        raise ValueError("world must be >= 1")
    total = int(off[-1]) if nchrom else 0
    bounds = [0]
    for k in range(1, world):
        target = total * k / world
        c = int(np.searchsorted(off[1:], target, side="left")) + 1   # first chromosome end >= target
        c = max(bounds[-1], min(nchrom, c))
        bounds.append(c)
    bounds.append(nchrom)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


def scan_range(shards: List[Tuple[int, int]], rank: int, prev_extra: bool) -> Tuple[int, int]:
    """Chromosomes rank `rank` actually scans: its shard, plus the preceding chromosome on the last
    non-empty rank when the final-block helper (Q9) is wanted."""
    lo, hi = shards[rank]
    last = max((r for r, (a, b) in enumerate(shards) if b > a), default=-1)
    if prev_extra and rank == last and lo > 0:
        lo -= 1
    return lo, hi


def _globalise(t: np.ndarray, slo: int, snp0: int) -> np.ndarray:
    """Local chromosome numbers and SNP indices of a rank's table -> global ones."""
    t = t.copy()
    t["chrom"] += slo
    live = (t["flags"] & L.W_EMPTY) == 0
    t["begin"][live] += snp0
    t["end"][live] += snp0
    return t


def merge_tables(tables: List[np.ndarray], shards: List[Tuple[int, int]], prev_extra: bool,
                 chrom_off: Sequence[int]) -> np.ndarray:
    """Concatenate per-rank record tables (each in its own local chromosome numbering and SNP
    indexing, as scanned over `scan_range`) into the global table a single-GPU plan over all
    chromosomes would emit."""
    off = np.asarray(chrom_off, dtype=np.int64)
    parts, extra = [], None
    last = max((r for r, (a, b) in enumerate(shards) if b > a), default=-1)
    for r, t in enumerate(tables):
        t = np.asarray(t, dtype=L.WINDOW_DTYPE)
        lo, hi = shards[r]
        slo, _ = scan_range(shards, r, prev_extra)
        if hi <= lo:
            continue
        body = _globalise(t[(t["flags"] & L.W_EXTRA) == 0], slo, int(off[slo]))
        body = body[body["chrom"] >= lo]          # the context chromosome belongs to its owner
        parts.append(body)
        if prev_extra and r == last:
            e = t[(t["flags"] & L.W_EXTRA) != 0]
            if len(e):
                e = _globalise(e, slo, int(off[slo]))
                e["wid"][(e["flags"] & L.W_EMPTY) == 0] += np.uint32(off[slo])   # helper: wid = SNP index
                extra = e
    out = np.concatenate(parts) if parts else np.zeros(0, dtype=L.WINDOW_DTYPE)
    if extra is not None:
        out = np.concatenate([out, extra])
    return out


def gather_tables(local: np.ndarray, world: int, device=None) -> List[np.ndarray]:
    """All-gather variable-length record tables over the default process group.  `device` is the
    torch device the exchange runs on (a GPU for RCCL, None / cpu for gloo)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cpu") if device is None else torch.device(device)
    raw = np.ascontiguousarray(local, dtype=L.WINDOW_DTYPE).view(np.uint8).reshape(-1, 64)
    n = torch.tensor([raw.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    m = max(ns) if ns else 0
    buf = torch.zeros((m, 64), dtype=torch.uint8, device=dev)
    if raw.shape[0]:
        buf[: raw.shape[0]] = torch.from_numpy(raw).to(dev)
    allb = torch.zeros((world * m, 64), dtype=torch.uint8, device=dev)
    if m:
        dist.all_gather_into_tensor(allb, buf)
    allb = allb.cpu().numpy().reshape(world, m, 64)
    return [allb[r, : ns[r]].copy().view(L.WINDOW_DTYPE).reshape(-1) for r in range(world)]


def window_starts(p, cfg) -> np.ndarray:
    """Global SNP indices where a window of the plan ``cfg`` starts (the cut candidates of a split):
    fixed-bp windows start where (pos-1)//ws or the chromosome changes; SNP-count windows every S
    SNPs from each chromosome's first (a chromosome's incomplete tail stays with its last window)."""
    from . import _lib as LL
    out = []
    for c in range(p.nchrom):
        lo, hi = int(p.chrom_off[c]), int(p.chrom_off[c + 1])
        if hi <= lo:
            continue
        if cfg.window_mode == LL.WINDOW_BP:
            w = (np.maximum(p.pos[lo:hi].astype(np.int64), 1) - 1) // int(cfg.window)
            out.append(lo + np.concatenate([[0], np.nonzero(np.diff(w))[0] + 1]))
        else:
            S = int(cfg.window)
            full = (hi - lo) // S
            out.append(lo + S * np.arange(max(full, 1)))
    return np.concatenate(out).astype(np.int64) if out else np.zeros(0, np.int64)


def split_points(p, cfg, world: int) -> List[int]:
    """Cuts 0 = c_0 <= c_1 <= ... <= c_world = n at window starts, c_k the one nearest k n / world:
    rank r scans SNPs [c_r, c_r+1) -- whole windows, chromosomes cut wherever that balances the
    SNPs.  With the Q9 helper (cfg.prev_extra) the last non-empty rank keeps >= 2 windows (the helper
    re-evaluates the window before the last one of the scan, against the last chromosome's
    background)."""
    n = p.n
    starts = window_starts(p, cfg)
    cuts = [0]
    for k in range(1, world):
        t = n * k / world
        j = int(np.searchsorted(starts, t))
        cand = [int(starts[i]) for i in (j - 1, j) if 0 <= i < len(starts)]
        c = min(cand, key=lambda x: abs(x - t)) if cand else n
        cuts.append(max(cuts[-1], min(c, n)))
    cuts.append(n)
    if cfg.prev_extra and len(starts) >= 2:
        last_ok = int(starts[-2])
        cuts = [0] + [min(c, last_ok) for c in cuts[1:-1]] + [n]
    return cuts


def _merge_split(tables, cuts, c0s, prev_extra, snp_window=0, chrom_off=None):
    """Rank tables (each numbered locally: chromosome 0 = the rank's first, SNPs from its cut) -> the
    global table: every rank's non-empty records in rank order (a window never spans two ranks),
    then the Q9 helper record of the last non-empty rank.  Empty bp slots are dropped (the post-pass
    skips them).  SNP-count windows (snp_window = S) of a part that starts inside a chromosome are
    renumbered from the windows before the cut (bp windows are numbered by position already)."""
    parts, extra = [], None
    for r, t in enumerate(tables):
        t = np.asarray(t, dtype=L.WINDOW_DTYPE).copy()
        if not len(t):
            continue
        live = (t["flags"] & L.W_EMPTY) == 0
        if snp_window:
            first = live & (t["chrom"] == 0)
            t["wid"][first] += np.uint32((cuts[r] - int(chrom_off[c0s[r]])) // snp_window)
        t["chrom"] += np.uint32(c0s[r])
        t["begin"][live] += np.uint32(cuts[r])
        t["end"][live] += np.uint32(cuts[r])
        is_x = (t["flags"] & L.W_EXTRA) != 0
        parts.append(t[live & ~is_x])
        if prev_extra and is_x.any():
            e = t[is_x]
            e["wid"][(e["flags"] & L.W_EMPTY) == 0] += np.uint32(cuts[r])   # the helper's wid: a SNP index
            extra = e
    out = np.concatenate(parts) if parts else np.zeros(0, dtype=L.WINDOW_DTYPE)
    return np.concatenate([out, extra]) if extra is not None else out


def _comm_device(device):
    import torch.distributed as dist
    return f"cuda:{device}" if dist.get_backend() == "nccl" else None


def _agree(err, size, world):
    """One collective: (any rank failed?, the largest `size` reported)."""
    import torch.distributed as dist
    got = [None] * world
    dist.all_gather_object(got, (err is not None, int(size)))
    return any(g[0] for g in got), max(g[1] for g in got)


def _allreduce_sum(v: np.ndarray, comm_device):
    import torch
    import torch.distributed as dist
    dev = torch.device("cpu") if comm_device is None else torch.device(comm_device)
    t = torch.from_numpy(np.ascontiguousarray(v, np.int64)).to(dev)
    dist.all_reduce(t)
    return t.cpu().numpy()


def hist_width(cfg) -> int:
    """Words of one chromosome's background row in the split exchange (L.bg_row_words: 2D bins,
    both unfolded 1D spectra, the inner 2D sum); 0 for a supplied background (nothing to exchange)."""
    return L.bg_row_words(cfg.n1p, cfg.n2p) if cfg.bg_mode == L.BG_PER_CHROM else 0


def whole_scan(split_scan):
    """The one-rank scan of a split-scan job factory: its own histograms are the totals."""
    def scan(sub, cfg, bg):
        job = split_scan(sub, cfg, bg)
        if hasattr(job, "whole"):
            return job.whole()
        return job.finish(job.partial())
    return scan


def _all_reduce_dev(buf):
    """Sum ``buf`` over the group where it lives: RCCL on the device (nccl); gloo reduces a host copy
    (the GPU tests' gloo groups: gloo's CUDA support is not relied on)."""
    import torch.distributed as dist
    if buf.is_cuda and dist.get_backend() != "nccl":
        h = buf.cpu()
        dist.all_reduce(h)
        buf.copy_(h)
    else:
        dist.all_reduce(buf)


def _all_gather_dev(out, world):
    """All-gather equal-size uint8 tables; the result on the host (the post-pass reads it there)."""
    import torch
    import torch.distributed as dist
    if out.is_cuda and dist.get_backend() != "nccl":
        out = out.cpu()
    g = torch.empty((world * out.shape[0], out.shape[1]), dtype=out.dtype, device=out.device)
    dist.all_gather_into_tensor(g, out)
    return g.cpu().numpy()


@contextlib.contextmanager
def _one_stream(eng, dev):
    """torch's ops on the exchange buffers, the collectives and the library's kernels ordered on ONE
    stream: a fresh torch stream made current and handed to the library; the engine's previous stream
    is restored on exit (the engine is shared per device: a caller that had handed it its own stream,
    as bench.py does, keeps it).  (Round 4 found the 2-rank test reading a NaN background once in
    several runs: the C API then took a NULL handle -- torch's default stream -- as the library's own
    non-blocking stream, unordered with the buffers' fill.  NULL is now the HIP null stream.)"""
    import torch
    s = torch.cuda.Stream(device=dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        prev = eng.set_stream(s.cuda_stream)
        try:
            yield s
        finally:
            s.synchronize()
            eng.set_stream(prev)


def _split_device(p, cfg, bg, split_scan, device, cuts, c0s, sub, c0, rank, world, last):
    """scan_records_split for jobs that exchange in HBM (engine.SplitJob).  Two collectives per scan,
    both on device buffers: ONE all-reduce of [every chromosome's background rows | per rank: failed,
    records] (each rank's part written by k_bg_rows_get; RCCL over xGMI), then ONE all-gather of the
    fixed-stride record tables, each followed by its rank's status row.  The host reads the small tail
    (to size the gather and to see failures) and the gathered table (the post-pass is sequential).
    Returns the merged table, or None when any rank failed (the caller falls back)."""
    import dataclasses

    import torch
    from .engine import Engine
    dev = torch.device(f"cuda:{device}")
    eng = Engine.get(device)
    W = hist_width(cfg)
    H = p.nchrom * W
    lo, hi = cuts[rank], cuts[rank + 1]
    job = None
    with _one_stream(eng, dev):   # kernels ordered with torch's / RCCL's ops
        try:
            buf = torch.zeros(H + 2 * world, dtype=torch.int64, device=dev)
            err, nrec = None, 0
            if hi > lo:
                try:
                    job = split_scan(sub, dataclasses.replace(cfg, prev_extra=bool(cfg.prev_extra) and rank == last), bg)
                    nrec = job.rows()
                    if W:
                        job.partial_dev(buf.data_ptr() + 8 * c0 * W, W)
                except Exception as e:  # noqa: BLE001  (every rank takes the fallback)
                    err = e
            buf[H + 2 * rank] = 1 if err is not None else 0
            buf[H + 2 * rank + 1] = nrec
            _all_reduce_dev(buf)
            STATS["allreduce"] += 1 if W else 0
            tail = buf[H:].cpu().numpy().reshape(world, 2)
            if tail[:, 0].any():
                return None
            rows = int(tail[:, 1].max())
            out = torch.zeros((rows + 1, 64), dtype=torch.uint8, device=dev)   # + this rank's status row
            if job is not None:
                try:
                    job.finish_dev(buf.data_ptr() + 8 * c0 * W if W else None, W, out.data_ptr())
                except Exception:  # noqa: BLE001
                    out[rows, 0] = 1
            g = _all_gather_dev(out, world).reshape(world, rows + 1, 64)
            if g[:, rows, 0].any():
                return None
            tables = [np.ascontiguousarray(g[r, : int(tail[r, 1])]).view(L.WINDOW_DTYPE).reshape(-1) for r in range(world)]
            return _merge_split(tables, cuts, c0s, bool(cfg.prev_extra),
                                int(cfg.window) if cfg.window_mode == L.WINDOW_SNPS else 0, p.chrom_off)
        finally:
            if job is not None:
                job.close()


def _rows_on_device(split_scan) -> bool:
    """Whether the jobs of ``split_scan`` exchange background rows in HBM: engine.SplitJob factories
    (``split_scan.device_rows``, or a factory whose jobs are SplitJob instances: ``split_scan.job_type``)."""
    from .engine import SplitJob
    if not (getattr(split_scan, "device_rows", False) or getattr(split_scan, "job_type", None) is SplitJob):
        return False
    try:
        import torch
        return torch.cuda.is_available()
    except ImportError:
        return False


def scan_records_split(p, cfg, bg, split_scan, device: int = 0, comm_device="auto") -> np.ndarray:
    """One scan of ``p`` split over the default process group at window boundaries (split_points):
    rank r scans SNPs [c_r, c_r+1) -- chromosomes cut wherever that balances the SNPs, so one
    chromosome spreads over all ranks.  With per-chromosome backgrounds every chromosome's histograms
    are the sum of its parts': between k_prep and the scan each rank's partial histograms are summed
    over the ranks (one all-reduce of int64 rows, SURVEY 8(e) collective (1)).

    ``split_scan(sub, cfg, bg)`` makes a rank's job over its part ``sub`` (chromosomes numbered from
    the part's first).  HIP jobs (``split_scan.device_rows``: engine.SplitJob) exchange in HBM
    (_split_device: the rows written and read back by kernels, RCCL on the device buffers).  Other jobs
    (the tests' oracle jobs) exchange on the host: ``job.partial()`` runs the histogram pass and returns
    the part's rows (int64 [nchrom, hist_width]; None without per-chromosome backgrounds), and
    ``job.finish(total)`` takes the summed rows, scans and returns the records.  Every rank returns the
    global record table (sfs2d.post reads it like one plan's).  When any rank fails, the whole scan is
    redone sharded by whole chromosomes (scan_records), which raises the error the reference raises on
    every rank (a chromosome's first bad SNP decides it, and it may sit in another rank's part)."""
    import dataclasses

    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    if comm_device == "auto":
        comm_device = _comm_device(device)
    cuts = split_points(p, cfg, world)
    lo, hi = cuts[rank], cuts[rank + 1]
    last = max((r for r in range(world) if cuts[r + 1] > cuts[r]), default=-1)
    sub, c0 = p.slice_snps(lo, hi)
    c0s = [p.slice_snps(cuts[r], cuts[r + 1])[1] for r in range(world)]
    if _rows_on_device(split_scan):
        out = _split_device(p, cfg, bg, split_scan, device, cuts, c0s, sub, c0, rank, world, last)
        if out is not None:
            STATS["split"] += 1
            return out
        STATS["fallback"] += 1
        return scan_records(p, cfg, bg, whole_scan(split_scan), device, comm_device)
    job, part, err = None, None, None
    if hi > lo:
        try:
            job = split_scan(sub, dataclasses.replace(cfg, prev_extra=bool(cfg.prev_extra) and rank == last), bg)
            part = job.partial()
        except Exception as e:  # noqa: BLE001  (every rank takes the fallback below)
            err = e
    failed, width = _agree(err, -1 if part is None else np.asarray(part).shape[1], world)
    local = np.zeros(0, dtype=L.WINDOW_DTYPE)
    if not failed:
        total = None
        if width > 0:
            g = np.zeros((p.nchrom, width), np.int64)
            if part is not None:
                g[c0:c0 + len(part)] = part
            total = _allreduce_sum(g.reshape(-1), comm_device).reshape(p.nchrom, width)
            STATS["allreduce"] += 1
        if job is not None:
            try:
                local = job.finish(None if total is None else total[c0:c0 + sub.nchrom])
            except Exception as e:  # noqa: BLE001
                err = e
        failed, _ = _agree(err, 0, world)
    if failed:
        # this rank's job (its uploaded part and plan) is released before the fallback re-uploads
        if job is not None and hasattr(job, "close"):
            job.close()
        STATS["fallback"] += 1
        return scan_records(p, cfg, bg, whole_scan(split_scan), device, comm_device)
    STATS["split"] += 1
    tables = gather_tables(local, world, comm_device)
    return _merge_split(tables, cuts, c0s, bool(cfg.prev_extra),
                        int(cfg.window) if cfg.window_mode == L.WINDOW_SNPS else 0, p.chrom_off)


def sharded_bg_hist(p, cfg, device: int = 0, chrom: int = -1):
    """calculate_2d_sfs / calculate_1d_sfs (twoDSFS_class.py:140-232, 398-444) over SNPs held by every
    rank of the default process group: rank r histograms the r-th of ``world`` contiguous SNP slices of
    chromosome ``chrom`` (-1: the whole data set) on its GPU into one int64 row (sfs2d_bg_hist_dev), and
    ONE all-reduce of [row | per rank: error bits] sums them (RCCL on the device buffer).  Every rank
    returns (h2d (n1+1, n2+1), unfolded h1a, unfolded h1b) as numpy int64, or raises what the
    single-GPU call raises: the error bits of all ranks are OR-ed, as one GPU's error word is (KeyError
    for counts above 2 * pop_size before the out-of-grid ValueError)."""
    import torch
    import torch.distributed as dist
    from .engine import Engine
    rank, world = dist.get_rank(), dist.get_world_size()
    lo_c, hi_c = (0, p.n) if chrom < 0 else (int(p.chrom_off[chrom]), int(p.chrom_off[chrom + 1]))
    span = hi_c - lo_c
    a, b = lo_c + span * rank // world, lo_c + span * (rank + 1) // world
    W = L.bg_row_words(cfg.n1p, cfg.n2p)
    on_dev = torch.cuda.is_available()
    dev = torch.device(f"cuda:{device}") if on_dev else torch.device("cpu")
    buf = torch.zeros(W + world, dtype=torch.int64, device=dev)
    code, err = 0, None
    if b > a:
        eng = Engine.get(device)
        try:
            with _one_stream(eng, dev):   # the histogram kernels ordered after buf's zero fill
                sub, _ = p.slice_snps(a, b)
                d = eng.upload(sub)
                try:
                    eng.bg_hist_dev(d, cfg, -1, buf.data_ptr())
                finally:
                    d.close()
        except KeyError:
            code = 1
        except L.Sfs2dError as e:
            code, err = (2, None) if e.code == L.E_GRID else (4, e)
        except Exception as e:  # noqa: BLE001  (every rank must reach the all-reduce: no RCCL hang)
            code, err = 4, e
    buf[W + rank] = code
    _all_reduce_dev(buf)
    h = buf.cpu().numpy()
    bits = int(np.bitwise_or.reduce(h[W:].astype(np.int64))) if world else 0
    if bits & 4:   # a failure other than the reference's count errors, on this rank or another
        if err is not None:
            raise err
        bad = [r for r in range(world) if int(h[W + r]) & 4]
        raise L.Sfs2dError(L.E_HIP, f"sharded background histogram failed on rank(s) {bad}")
    if bits & 1:
        raise KeyError("allele count above 2*pop_size (reference: KeyError in calculate_1d_sfs)")
    if bits & 2:
        raise L.Sfs2dError(L.E_GRID, "folded 2D bin outside the (2n1+1)x(2n2+1) grid")
    n1, n2 = 2 * cfg.n1p, 2 * cfg.n2p
    nb = (n1 + 1) * (n2 + 1)
    return h[:nb].reshape(n1 + 1, n2 + 1), h[nb:nb + n1 + 1], h[nb + n1 + 1:nb + n1 + n2 + 2]


def scan_records(p, cfg, bg, scan_local, device: int = 0, comm_device="auto") -> np.ndarray:
    """One scan of ``p`` (ScanConfig ``cfg``, supplied background ``bg`` or None) sharded over the
    default process group: this rank scans its chromosome range with ``scan_local(sub, cfg, bg)``
    (the HIP scan of one GPU), the tables are all-gathered and merged.  Every rank returns the global
    record table (what one plan over all of ``p`` emits: slots in chromosome order, the Q9 helper
    record last when ``cfg.prev_extra``)."""
    import dataclasses

    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    shards = shard_chromosomes(p.chrom_off, world)
    pe = bool(cfg.prev_extra)
    lo, hi = scan_range(shards, rank, pe)
    last = max((r for r, (a, b) in enumerate(shards) if b > a), default=-1)
    local = np.zeros(0, dtype=L.WINDOW_DTYPE)
    err = None
    if shards[rank][1] > shards[rank][0]:
        sub = p.subset_chroms(range(lo, hi))
        try:
            local = scan_local(sub, dataclasses.replace(cfg, prev_extra=pe and rank == last), bg)
        except Exception as e:  # noqa: BLE001  (raised on every rank below, not left to hang the gather)
            err = e
    _raise_collective(err, world)
    if comm_device == "auto":
        comm_device = _comm_device(device)
    tables = gather_tables(local, world, comm_device)
    return merge_tables(tables, shards, pe, p.chrom_off)


def _raise_collective(err, world):
    """A rank's scan error (e.g. KeyError for counts above the sample size, found by the rank that
    holds the SNP) raised on every rank, the lowest failing rank's: no rank is left waiting in the
    gather."""
    import builtins

    import torch.distributed as dist
    got = [None] * world
    dist.all_gather_object(got, None if err is None else (type(err).__name__, str(err.args[0]) if err.args else ""))
    first = next((g for g in got if g is not None), None)
    if first is None:
        return
    if err is not None and (type(err).__name__, str(err.args[0]) if err.args else "") == first:
        raise err
    t = getattr(builtins, first[0], None)
    if isinstance(t, type) and issubclass(t, Exception):
        raise t(first[1])
    raise L.Sfs2dError(L.E_HIP, f"{first[0]} on another rank: {first[1]}")


def combined_scan_sharded(packed, window_size: int, n1p: int, n2p: int, rank: int, world: int,
                          device: int = 0, comm_device=None, fold: bool = True) -> Optional[dict]:
    """combined_scan (twoDSFS_class.py:787-991) over `world` GPUs: every rank holds the packed SNPs
    on the host, uploads and scans its chromosome range; rank 0 returns the reference's result
    dict, the other ranks None."""
    from . import post
    from .engine import Engine, ScanConfig
    shards = shard_chromosomes(packed.chrom_off, world)
    lo, hi = scan_range(shards, rank, True)
    local = np.zeros(0, dtype=L.WINDOW_DTYPE)
    if shards[rank][1] > shards[rank][0]:
        sub = packed.subset_chroms(range(lo, hi))
        eng = Engine.get(device)
        dev = eng.upload(sub)
        local = eng.scan(dev, ScanConfig(n1p=n1p, n2p=n2p, fold=fold, window=window_size,
                                         prev_extra=(rank == max(r for r, (a, b) in enumerate(shards) if b > a))))
        dev.close()
    tables = gather_tables(local, world, comm_device)
    if rank != 0:
        return None
    recs = merge_tables(tables, shards, True, packed.chrom_off)
    return post.combined_scan(recs, packed, window_size, post.num_slots(recs))
