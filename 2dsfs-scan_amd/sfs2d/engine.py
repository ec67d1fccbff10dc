"""Host-side runtime over the C ABI: contexts, resident data sets, scan plans.

One ``Engine`` per GPU (one process per GPU for multi-GPU runs).  A ``DeviceData`` is a packed
SNP set resident in HBM; a ``Plan`` holds everything that depends on (data, scan parameters)
and replays the kernels.  See include/sfs2d.h for the contract.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib as L
from .pack import PackedSNPs


@dataclass
class ScanConfig:
    n1p: int
    n2p: int
    fold: bool = True
    window_mode: int = L.WINDOW_BP
    window: int = 20000
    bg_mode: int = L.BG_PER_CHROM
    ann_want: int = -1
    start_position: Optional[int] = None
    end_position: Optional[int] = None
    prev_extra: bool = False
    fst: bool = False          # also compute Hudson's Fst per window slot (Plan.read_fst)
    scan_wgs_per_cu: int = 0   # cap on scan workgroups per CU (0: all that fit; see sfs2d_params)

    def params(self) -> L.Params:
        p = L.Params()
        p.n1p, p.n2p, p.fold = int(self.n1p), int(self.n2p), 1 if self.fold else 0
        p.window_mode, p.window, p.bg_mode = int(self.window_mode), int(self.window), int(self.bg_mode)
        p.ann_want = int(self.ann_want)
        # Python ints of any size: clamp into the int64 range the kernel compares against
        clamp = lambda v: max(-(1 << 62), min(1 << 62, int(v)))
        p.has_start = 0 if self.start_position is None else 1
        p.start_pos = 0 if self.start_position is None else clamp(self.start_position)
        p.has_end = 0 if self.end_position is None else 1
        p.end_pos = 0 if self.end_position is None else clamp(self.end_position)
        p.flags = (L.F_PREV_EXTRA if self.prev_extra else 0) | (L.F_FST if self.fst else 0)
        p.scan_wgs_per_cu = int(self.scan_wgs_per_cu)
        return p


class Engine:
    _cache = {}

    def __init__(self, device: int = 0):
        self.lib = L.lib()
        self.device = device
        h = C.c_void_p()
        rc = self.lib.sfs2d_ctx_create(device, C.byref(h))
        if rc != 0:
            raise L.Sfs2dError(rc, f"cannot create a HIP context on device {device} (no MI355X visible?)")
        self.h = h
        self.stream = None   # the ctx's own stream (set_stream)

    @classmethod
    def get(cls, device: int = 0) -> "Engine":
        e = cls._cache.get(device)
        if e is None:
            e = cls(device)
            cls._cache[device] = e
        return e

    def check(self, rc):
        if rc != 0:
            msg = self.lib.sfs2d_last_error(self.h).decode()
            if rc == L.E_KEY:
                raise KeyError(msg)
            raise L.Sfs2dError(rc, msg)

    def set_stream(self, stream_handle: Optional[int]):
        """Enqueue the library's work on the HIP stream ``stream_handle``: any handle, 0 included (the
        HIP null stream -- torch's default stream -- ordered with the process's blocking streams);
        None: the ctx's own non-blocking stream (sfs2d_ctx_use_own_stream), which nothing orders
        against the caller's streams.  Returns the previous setting (for restore)."""
        prev = self.stream
        if stream_handle is None:
            self.check(self.lib.sfs2d_ctx_use_own_stream(self.h))
        else:
            self.check(self.lib.sfs2d_ctx_set_stream(self.h, C.c_void_p(int(stream_handle)) if int(stream_handle) else None))
        self.stream = stream_handle
        return prev

    def stream_handle(self) -> int:
        """The HIP stream handle the library currently enqueues on (sfs2d_ctx_get_stream): the ctx's own
        stream after construction or ``set_stream(None)``, 0 for the null stream."""
        s = C.c_void_p()
        self.check(self.lib.sfs2d_ctx_get_stream(self.h, C.byref(s)))
        return int(s.value or 0)

    def upload(self, p: PackedSNPs) -> "DeviceData":
        return DeviceData(self, p)

    def wrap_device(self, d_counts: int, d_pos: int, d_ann: Optional[int], n: int, chrom_off: np.ndarray,
                    chrom_last_pos: np.ndarray) -> "DeviceData":
        return DeviceData(self, None, (d_counts, d_pos, d_ann, n, chrom_off, chrom_last_pos))

    def synth_sims(self, seed: int, generation: int, n_rep: int, n_win: int, window_bp: int, n1p: int, n2p: int,
                   win_counts: np.ndarray, mt1: np.ndarray, mt2: np.ndarray) -> "DeviceData":
        """BASELINE config 4: n_rep replicate chromosomes generated in HBM (sfs2d_data_synth_sims)."""
        sp = L.SynthParams(seed=seed, generation=generation, n_replicates=n_rep, n_windows=n_win,
                           window_bp=window_bp, n1p=n1p, n2p=n2p)
        wc = np.ascontiguousarray(win_counts, np.uint16)
        m1 = np.ascontiguousarray(mt1, np.uint32)
        m2 = np.ascontiguousarray(mt2, np.uint32)
        h = C.c_void_p()
        self.check(self.lib.sfs2d_data_synth_sims(self.h, C.byref(sp), L.ptr(wc), L.ptr(m1), len(m1), L.ptr(m2),
                                                  len(m2), C.byref(h)))
        return DeviceData(self, None, dev=h)

    def bg_hist(self, data: "DeviceData", cfg: ScanConfig, chrom: int = -1):
        n1, n2 = 2 * cfg.n1p, 2 * cfg.n2p
        h2 = np.zeros((n1 + 1) * (n2 + 1), np.int64)
        h1a = np.zeros(n1 + 1, np.int64)
        h1b = np.zeros(n2 + 1, np.int64)
        prm = cfg.params()
        self.check(self.lib.sfs2d_bg_hist(self.h, data.h, C.byref(prm), int(chrom), L.ptr(h2), L.ptr(h1a),
                                          L.ptr(h1b)))
        return h2.reshape(n1 + 1, n2 + 1), h1a, h1b

    def bg_hist_dev(self, data: "DeviceData", cfg: ScanConfig, chrom: int, row_ptr: int):
        """sfs2d_bg_hist_dev: the histograms as one int64 row (L.bg_row_words) at device address
        ``row_ptr``, enqueued on the engine's stream (synchronises to report count errors)."""
        prm = cfg.params()
        self.check(self.lib.sfs2d_bg_hist_dev(self.h, data.h, C.byref(prm), int(chrom), C.c_void_p(row_ptr)))

    def plan(self, data: "DeviceData", cfg: ScanConfig) -> "Plan":
        return Plan(self, data, cfg)

    def scan(self, data: "DeviceData", cfg: ScanConfig, bg=None) -> np.ndarray:
        """One-shot scan; returns the window records (numpy structured array, WINDOW_DTYPE)."""
        pl = Plan(self, data, cfg)
        try:
            if cfg.bg_mode == L.BG_SUPPLIED:
                pl.set_background(*bg)
            pl.run()
            pl.check()
            return pl.read()
        finally:
            pl.close()


class DeviceData:
    def __init__(self, eng: Engine, p: Optional[PackedSNPs], dev=None):
        self.eng = eng
        self.h = C.c_void_p()
        if isinstance(dev, C.c_void_p):   # a handle the library already created (sfs2d_data_synth_sims)
            self.packed = None
            self.h = dev
            return
        if p is not None:
            self.packed = p
            off = np.ascontiguousarray(p.chrom_off, np.int64)
            eng.check(eng.lib.sfs2d_data_upload(eng.h, L.ptr(p.counts), L.ptr(p.pos), L.ptr(p.ann_id), p.n,
                                                L.ptr(off), p.nchrom, C.byref(self.h)))
        else:
            d_counts, d_pos, d_ann, n, chrom_off, last_pos = dev
            self.packed = None
            off = np.ascontiguousarray(chrom_off, np.int64)
            lp = np.ascontiguousarray(last_pos, np.uint32)
            eng.check(eng.lib.sfs2d_data_wrap_device(eng.h, C.c_void_p(d_counts), C.c_void_p(d_pos),
                                                     C.c_void_p(d_ann) if d_ann else None, int(n), L.ptr(off),
                                                     L.ptr(lp), len(off) - 1, C.byref(self.h)))

    def read(self, n: int):
        """(counts, pos) of the data set back on the host (n = its SNP count)."""
        c = np.zeros(n, np.uint32)
        p = np.zeros(n, np.uint32)
        self.eng.check(self.eng.lib.sfs2d_data_read(self.h, L.ptr(c), L.ptr(p), int(n)))
        return c, p

    def close(self):
        if self.h:
            self.eng.lib.sfs2d_data_free(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Plan:
    def __init__(self, eng: Engine, data: DeviceData, cfg: ScanConfig, base: "Optional[Plan]" = None):
        self.eng, self.data, self.cfg, self.base = eng, data, cfg, base
        self.h = C.c_void_p()
        self.attached = []
        prm = cfg.params()
        if base is None:
            eng.check(eng.lib.sfs2d_plan_create(eng.h, data.h, C.byref(prm), C.byref(self.h)))
        else:
            eng.check(eng.lib.sfs2d_plan_attach(base.h, C.byref(prm), C.byref(self.h)))
            base.attached.append(self)
        self.nrec = int(eng.lib.sfs2d_plan_num_records(self.h))

    def attach(self, cfg: ScanConfig) -> "Plan":
        """A plan scanned from this plan's k_prep pass (another window size / SNP-count windows):
        run this (base) plan, then read the attached one (sfs2d_plan_attach)."""
        return Plan(self.eng, self.data, cfg, base=self)

    def set_background(self, bg2d, bg1a, bg1b):
        n1p, n2p = self.cfg.n1p, self.cfg.n2p
        b2 = np.ascontiguousarray(np.asarray(bg2d, np.float64).reshape(-1))
        b1 = np.ascontiguousarray(np.asarray(bg1a, np.float64).reshape(-1)[: n1p + 1])
        b1b = np.ascontiguousarray(np.asarray(bg1b, np.float64).reshape(-1)[: n2p + 1])
        if b2.size != (2 * n1p + 1) * (2 * n2p + 1) or b1.size != n1p + 1 or b1b.size != n2p + 1:
            raise ValueError("background arrays have the wrong size")
        self.eng.check(self.eng.lib.sfs2d_plan_set_background(self.h, L.ptr(b2), L.ptr(b1), L.ptr(b1b)))

    def run(self, out_dev_ptr: Optional[int] = None, phase: int = 0):
        self.eng.check(self.eng.lib.sfs2d_plan_run_phase(self.h, phase,
                                                         C.c_void_p(out_dev_ptr) if out_dev_ptr else None))

    def read_fst(self) -> np.ndarray:
        """Fst of the last run per window slot (NaN = no qualifying SNP / empty slot)."""
        dptr, n = C.c_void_p(), C.c_int64()
        self.eng.check(self.eng.lib.sfs2d_plan_fst_buffer(self.h, C.byref(dptr), C.byref(n)))
        out = np.zeros(n.value, dtype=np.float64)
        self.eng.check(self.eng.lib.sfs2d_plan_fst_read(self.h, out.ctypes.data if n.value else None, n.value))
        return out

    def set_fst_out(self, dev_ptr: Optional[int]):
        """Write the Fst of the following runs to the device buffer at ``dev_ptr`` (>= nslots float64; None:
        the plan's own buffer, which read_fst reads) -- sfs2d_plan_set_fst_out."""
        self.eng.check(self.eng.lib.sfs2d_plan_set_fst_out(self.h, C.c_void_p(dev_ptr) if dev_ptr else None))

    def run_many(self, nruns: int, out_dev_ptr: Optional[int] = None):
        """Enqueue `nruns` back-to-back runs from C (no Python between runs)."""
        self.eng.check(self.eng.lib.sfs2d_plan_run_many(self.h, int(nruns),
                                                        C.c_void_p(out_dev_ptr) if out_dev_ptr else None))

    @staticmethod
    def run_streams(plans, streams, nruns: int, out_dev_ptrs=None):
        """Enqueue `nruns` runs round-robin over distinct plans of one engine, run i on
        streams[i % len(plans)] (sfs2d_plan_run_streams: independent scans overlap across the streams).
        Entries are HIP stream handles, 0 = the HIP null stream (as in Engine.set_stream); None = the
        stream the engine currently enqueues on (Engine.stream_handle), so that ``read()`` / ``check()``,
        which synchronise that stream, see those runs finished."""
        k = len(plans)
        eng = plans[0].eng
        cur = eng.stream_handle() if any(s is None for s in streams) else 0
        ph = (C.c_void_p * k)(*[p.h.value for p in plans])
        sh = (C.c_void_p * k)(*[(cur if s is None else int(s)) or None for s in streams])
        oh = (C.c_void_p * k)(*[o or None for o in out_dev_ptrs]) if out_dev_ptrs else None
        eng.check(eng.lib.sfs2d_plan_run_streams(ph, sh, oh, k, int(nruns)))

    @staticmethod
    def graph(plans, streams, nruns: int, out_dev_ptrs=None):
        """``run_streams(plans, streams, nruns, out_dev_ptrs)`` captured once into a HIP graph
        (sfs2d_graph_create, one graph per stream): ``RunGraph.launch(n)`` replays it n times, one
        hipGraphLaunch per stream and replay.
        `nruns` a multiple of 2 * len(plans); streams non-null HIP stream handles."""
        k = len(plans)
        eng = plans[0].eng
        if any(not s for s in streams):
            raise ValueError("Plan.graph: non-null stream handles")
        ph = (C.c_void_p * k)(*[p.h.value for p in plans])
        sh = (C.c_void_p * k)(*[int(s) for s in streams])
        oh = (C.c_void_p * k)(*[o or None for o in out_dev_ptrs]) if out_dev_ptrs else None
        h = C.c_void_p()
        eng.check(eng.lib.sfs2d_graph_create(ph, sh, oh, k, int(nruns), C.byref(h)))
        return RunGraph(eng, h, list(plans), int(nruns))

    def check(self):
        self.eng.check(self.eng.lib.sfs2d_plan_check(self.h))

    def read(self) -> np.ndarray:
        out = np.zeros(self.nrec, dtype=L.WINDOW_DTYPE)
        n = C.c_int64()
        self.eng.check(self.eng.lib.sfs2d_plan_read(self.h, L.ptr(out), self.nrec, C.byref(n)))
        return out

    def bg_buffer(self):
        p = C.c_void_p()
        nb = C.c_int64()
        self.eng.check(self.eng.lib.sfs2d_plan_bg_buffer(self.h, C.byref(p), C.byref(nb)))
        return p.value, nb.value

    def time(self, iters: int = 10):
        v = [C.c_double() for _ in range(4)]
        self.eng.check(self.eng.lib.sfs2d_plan_time(self.h, iters, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def grids(self):
        """(k_prep threads, scan kernel threads) per launch: rocprofv3's Grid_Size of each kernel."""
        a, b = C.c_int64(), C.c_int64()
        self.eng.check(self.eng.lib.sfs2d_plan_grids(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def scan_kernel(self) -> str:
        """Name of the scan kernel this plan launches (the prefix of its rocprofv3 kernel name)."""
        return self.eng.lib.sfs2d_plan_scan_kernel(self.h).decode()

    def stats(self) -> int:
        v = C.c_uint32()
        self.eng.check(self.eng.lib.sfs2d_plan_stats(self.h, C.byref(v)))
        return int(v.value)

    def set_timing(self, max_runs: int, every: int = 1, kernels: int = 7):
        """Record HIP events around each kernel of every `every`-th following run (<= max_runs samples);
        `kernels`: bit 0 k_prep, bit 1 k_bg_slice, bit 2 the scan kernel (the others read 0)."""
        self.eng.check(self.eng.lib.sfs2d_plan_set_timing_kernels(self.h, int(max_runs), int(every), int(kernels)))

    def timing_read(self):
        n = C.c_int()
        v = [C.c_double() for _ in range(3)]
        self.eng.check(self.eng.lib.sfs2d_plan_timing_read(self.h, C.byref(n), *[C.byref(x) for x in v]))
        return n.value, tuple(x.value for x in v)

    def close(self):
        if self.h:
            for a in self.attached:   # destroyed by the library together with this base
                a.h = C.c_void_p()
            self.attached = []
            if self.base is not None and self in self.base.attached:
                self.base.attached.remove(self)
            self.eng.lib.sfs2d_plan_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RunGraph:
    """A captured run sequence (Plan.graph / sfs2d_graph_*): `runs` plan runs per launch."""

    def __init__(self, eng, h, plans, runs):
        self.eng, self.h, self.plans, self.runs = eng, h, plans, runs

    def launch(self, n: int = 1):
        """Replay n times, on the capture streams (each replay after the stream's earlier work)."""
        self.eng.check(self.eng.lib.sfs2d_graph_launch(self.h, int(n)))

    def close(self):
        if self.h:
            self.eng.lib.sfs2d_graph_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SplitJob:
    """A rank's part of a scan split over ranks at window boundaries (sfs2d.dist.scan_records_split):
    its SNPs uploaded and one plan.  The exchange stays in HBM: ``partial_dev`` runs k_prep alone
    (phase 1) and writes this part's per-chromosome background histograms as int64 rows into a device
    buffer (sfs2d_plan_bg_rows_dev); after the ranks' all-reduce of that buffer (RCCL), ``finish_dev``
    writes the summed rows back (sfs2d_plan_bg_rows_set_dev), runs tables + scan (phase 2) into a device
    record buffer and checks the run.  ``whole`` is the one-rank scan (its own histograms are the totals).
    Everything is enqueued on the engine's stream: the caller sets it to the stream its collectives are
    ordered on (torch's current stream)."""

    device_rows = True

    def __init__(self, eng: Engine, sub: PackedSNPs, cfg: ScanConfig, bg=None):
        self.eng, self.cfg, self.nchrom = eng, cfg, sub.nchrom
        self.dev = eng.upload(sub)
        self.pl = None
        try:
            self.pl = Plan(eng, self.dev, cfg)
            if cfg.bg_mode == L.BG_SUPPLIED:
                self.pl.set_background(*bg)
        except Exception:
            self.close()
            raise

    def rows(self) -> int:
        """Records the scan writes (window slots, + the Q9 helper)."""
        return self.pl.nrec

    def partial_dev(self, rows_ptr: int, stride: int):
        """k_prep alone; this part's background histograms into ``rows_ptr`` (int64, row c at
        rows_ptr + 8 * c * stride).  Nothing to do for a supplied background."""
        if self.cfg.bg_mode != L.BG_PER_CHROM:
            return
        self.pl.run(phase=1)
        self.eng.check(self.eng.lib.sfs2d_plan_bg_rows_dev(self.pl.h, C.c_void_p(rows_ptr), int(stride)))

    def finish_dev(self, rows_ptr: Optional[int], stride: int, out_ptr: int):
        """The summed rows back, the scan into ``out_ptr`` (device, rows() records), errors raised."""
        try:
            if self.cfg.bg_mode == L.BG_PER_CHROM:
                self.eng.check(self.eng.lib.sfs2d_plan_bg_rows_set_dev(self.pl.h, C.c_void_p(rows_ptr), int(stride)))
                self.pl.run(out_ptr, phase=2)
            else:
                self.pl.run(out_ptr)
            self.pl.check()
        finally:
            self.close()

    def whole(self) -> np.ndarray:
        """The part scanned on its own (one rank: its histograms are the totals); host records."""
        try:
            self.pl.run()
            self.pl.check()
            return self.pl.read()
        finally:
            self.close()

    def close(self):
        if self.pl is not None:
            self.pl.close()
            self.pl = None
        if self.dev is not None:
            self.dev.close()
            self.dev = None

