#!/usr/bin/env python3
"""Benchmark: genomic windows/s of the 2D-SFS composite-likelihood scan (BASELINE.json metric).

Workload (BASELINE configs[1]): one synthetic chromosome of 1e6 SNPs per GPU (SURVEY 8d
generator, seed 12345 + rank), n1 = n2 = 50 haploid (pop_size 25/25), 20 kb fixed-bp windows,
each chromosome its own background (combined_scan semantics).  A step = one full scan pass over
the HBM-resident packed SNPs: background histograms + window segmentation (K1), background
tables (K2), window scan (K3) -> device-resident 64-B window records.  Consecutive passes are
independent: they go round-robin over --streams plans (default 3), each on its own HIP stream, so
one pass's latency-bound kernels overlap the next one's (sfs2d_plan_run_streams).  The timed loop
is the same at every N (weak scaling: each rank its own chromosome, no data-path collective); with
N > 1 ranks the timed region ends with one RCCL all-gather of every rank's final window table.

`--gpus N` with no launcher: this script starts the N rank processes itself (before touching the
GPU) and exits with their status; under torchrun, WORLD_SIZE must equal N, and a box with fewer
than N GPUs fails instead of reporting fewer.

Prints ONE JSON line on rank 0.  `roofline` is for the dominant kernel (K3) from HIP events in its
dispatch packets, on the stream it runs on (with overlapped passes: in a single-stream pass right
after the timed steps, whose durations agree with rocprofv3's kernel trace; the contended interval
of the timed steps is `ms_timed_region`); `roofline_hbm` repeats the measurement
on a >= 400 MB stream (BASELINE config 3 at 1 GPU: 32 x 1.5625e6 SNPs) that does not fit the
256 MB Infinity Cache.  `cpu_baseline` times the CPU oracle (a numpy/scipy restatement of the
reference's dense per-window algorithm, 1 core) on a bounded sample of the same stream.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "2dsfs-scan_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
N_SNP = 1_000_000
POP = 25
WS = 20000


def algorithmic_bytes(n_snp, n_slots, n_win, which):
    """Bytes each kernel must move (DESIGN.md "Kernels"), counted from its inputs and outputs.

    k_prep ("k1"): reads counts + positions (8 B/SNP), writes the window slot table (8 B/window) (a
    counts plan stores no per-SNP bins).  k_scan_w ("k3"): reads the counts (4 B/SNP), the slot
    record (8 B/slot) and the slot's Fst sums (16 B/slot), writes one 64-B record and one 8-B Fst
    value per slot.  "pipeline": SURVEY.md 8(d)'s per-unit figure for a whole step -- 8 B/SNP for
    the scan pass + 4 B/SNP for the background pass over the same stream + 64 B per output window."""
    if which == "k3":
        return 4 * n_snp + (8 + 16 + 64 + 8) * n_slots
    if which == "k1":
        return 8 * n_snp + 8 * n_win
    if which == "pipeline":
        return 12 * n_snp + 64 * n_win
    raise ValueError(which)


def pmc_traffic(kernel, grid):
    """HBM bytes per launch of `kernel` at `grid` threads from the committed rocprofv3 --pmc passes
    of this bench command (tools/pmc_bench.sh -> profiles/pmc_bench.json: FETCH_SIZE x 2 per the
    gfx950 correction of MI355X_MICROARCH.md, + WRITE_SIZE; separate passes).  None when absent."""
    path = os.path.join(REPO, "profiles", "pmc_bench.json")
    try:
        with open(path) as fh:
            d = json.load(fh)
    except (OSError, ValueError):
        return None, None
    for r in d.get("kernels", []):
        if r.get("kernel", "").startswith(kernel) and int(r.get("grid", -1)) == int(grid):
            return r["read_bytes"] + r["write_bytes"], d.get("source", path)
    return None, None


def cpu_baseline(p):
    """The CPU baseline on this box's host cores: the C restatement of the oracle (oracle/sfs_oracle_c.c,
    the reference's dense per-window algorithm, OpenMP over windows; test infrastructure, pinned to
    the numpy oracle) over the whole rank-0 config-2 stream, repeated for >= 3 s; beside it the numpy
    oracle itself (dense grids + scipy multinomial.logpmf, as the reference computes them) on one core
    over the same stream."""
    from oracle import sfs_oracle as O
    from oracle import sfs_oracle_c as OC
    threads = min(16, os.cpu_count() or 1)   # the box's CPU share (OMP_NUM_THREADS is 16 there)
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        threads = min(threads, int(os.environ["OMP_NUM_THREADS"]))
    OC.scan_bp(p, WS, POP, POP, threads)   # warm
    reps, t0 = 0, time.perf_counter()
    while True:
        r = OC.scan_bp(p, WS, POP, POP, threads)
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= 3.0:
            break
    nwin = len(r["b"])
    cfg = O.Cfg(POP, POP)
    t1 = time.perf_counter()
    res = O.combined_scan(p, WS, cfg)
    dt1 = time.perf_counter() - t1
    return {"value": nwin * reps / dt, "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"the full rank-0 config-2 stream ({p.n} SNPs, {nwin} windows) x {reps} in {dt:.1f} s: "
                      "oracle/sfs_oracle_c.c (the reference's dense per-window grids and scipy's logpmf "
                      f"closed form, numpy's pairwise p-sums), OpenMP over windows on {threads} host threads",
            "numpy_oracle_1core": {"value": len(res) / dt1, "unit": "windows/s", "cores": 1,
                                   "sample": f"oracle/sfs_oracle.combined_scan on the same stream ({dt1:.1f} s)"}}


def end_to_end(n_rec=1_000_000, nchrom=8, seed=3):
    """The reference script's job end to end (twoDSFS_class.py:1910-2040: make_data_dict_vcf, then
    combined_scan at 20 kb and 500 kb and scan_perChr_bySNPs at 500 SNPs, save_csv_stats) as this
    framework runs it (python -m sfs2d): a synthetic BGZF VCF of n_rec records x 32 samples (18 uv +
    14 bv, the reference's popmap shape) -> native ingest -> packed upload -> one k_prep pass + three
    scans (multi_scan) -> three CSVs.  Wall time from the file on disk to the CSVs written."""
    import tempfile
    import zlib
    import struct
    from sfs2d import cli
    rng = np.random.default_rng(seed)
    samples = [f"S{i}" for i in range(32)]
    d = tempfile.mkdtemp(prefix="sfs2d_e2e_")
    vcf, pm = os.path.join(d, "synth.vcf.gz"), os.path.join(d, "popmap.txt")
    with open(pm, "w") as fh:
        fh.write("".join(f"{x}\t{'uv' if i < 18 else 'bv'}\n" for i, x in enumerate(samples)))
    t0 = time.perf_counter()
    gts = np.frombuffer(b"0/0\t0/1\t1/1\t./.\t1/0\t", dtype="S4")
    g = gts[rng.choice(5, size=(n_rec, 32), p=[0.5, 0.2, 0.15, 0.05, 0.1])].view(np.uint8).reshape(n_rec, 128)
    g[:, -1] = ord("\n")
    per = n_rec // nchrom
    pos = np.concatenate([np.cumsum(rng.integers(1, 110, per)) for _ in range(nchrom)] +
                         [np.cumsum(rng.integers(1, 110, n_rec - per * nchrom))])
    chrom = [f"chr{min(i // per, nchrom - 1) + 1}" for i in range(n_rec)]
    pre = [f"{c}\t{q}\t.\tA\tG\t.\tPASS\tPR\tGT\t".encode() for c, q in zip(chrom, pos.tolist())]
    body = b"".join(a + b for a, b in zip(pre, (bytes(r) for r in g)))
    head = ("##fileformat=VCFv4.2\n#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples) + "\n").encode()
    text = head + body
    out = bytearray()
    for i in range(0, len(text), 65280):   # BGZF blocks (SAM spec 4.1), then the EOF block
        chunk = text[i:i + 65280]
        c = zlib.compressobj(1, zlib.DEFLATED, -15)
        cd = c.compress(chunk) + c.flush()
        out += (b"\x1f\x8b\x08\x04" + b"\x00" * 4 + b"\x00\xff" + struct.pack("<H", 6) + b"BC" +
                struct.pack("<HH", 2, 18 + len(cd) + 8 - 1) + cd + struct.pack("<II", zlib.crc32(chunk), len(chunk)))
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    with open(vcf, "wb") as fh:
        fh.write(out)
    t_gen = time.perf_counter() - t0
    args = [vcf, pm, "--window", "20000", "--window", "500000", "--snp-window", "500",
            "--out-prefix", os.path.join(d, "stats")]
    import contextlib
    import io
    cli.main(args)   # warm: library loads, first HIP context / plan allocations
    err = io.StringIO()
    t0 = time.perf_counter()
    with contextlib.redirect_stderr(err):
        outs = cli.main(args)
    wall = time.perf_counter() - t0
    rows = sum(max(0, sum(1 for _ in open(o)) - 1) for o in outs)
    stages = [ln for ln in err.getvalue().splitlines() if ln.startswith(("ingest", "multi_scan"))]
    for f in os.listdir(d):
        os.remove(os.path.join(d, f))
    os.rmdir(d)
    return {"wall_s": wall, "records": n_rec, "records_per_s": n_rec / wall, "csv_rows": rows,
            "vcf_bytes": len(out), "stages": stages, "generate_s": t_gen,
            "workload": f"synthetic BGZF VCF, {n_rec} records x 32 samples (18 uv + 14 bv), {nchrom} chromosomes; "
                        "python -m sfs2d --window 20000 --window 500000 --snp-window 500 (the reference "
                        "script's three scans) from the file on disk to the three CSVs written, second run"}


def hbm_stream_roofline(eng, steps=5):
    """BASELINE config 3 on one GPU (5e7 SNPs, 32 chromosomes, ~600 MB read): past the MALL."""
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(32, 1_562_500, POP, POP, seed=777)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=POP, n2p=POP, window=WS, fst=True))
    pl.run()
    pl.check()
    pl.set_timing(steps, every=2)
    pl.run_many(2 * steps)
    nr, (k1, k2, k3) = pl.timing_read()
    pl.set_timing(0)
    pl.check()
    t0 = time.perf_counter()
    pl.run_many(4 * steps)
    pl.check()
    wall = (time.perf_counter() - t0) / (4 * steps)   # per run, back to back (gaps included)
    recs = pl.read()
    nwin = int(((recs["flags"] & 0x80000000) == 0).sum())
    b3 = algorithmic_bytes(p.n, pl.nrec, nwin, "k3")
    b1 = algorithmic_bytes(p.n, pl.nrec, nwin, "k1")
    bp = algorithmic_bytes(p.n, pl.nrec, nwin, "pipeline")
    out = {"bound": "hbm", "achieved": b3 / (k3 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": b3 / (k3 * 1e-3) / 1e9 / HBM_PEAK_GBS, "kernel": "k_scan_w", "ms": k3,
           "k1_GBs": b1 / (k1 * 1e-3) / 1e9, "k1_frac": b1 / (k1 * 1e-3) / 1e9 / HBM_PEAK_GBS, "k1_ms": k1,
           "k2_ms": k2,
           "serial": {"pipeline_GBs": bp / wall / 1e9, "pipeline_frac": bp / wall / 1e9 / HBM_PEAK_GBS,
                      "pipeline_ms": wall * 1e3, "windows_per_s": nwin / wall,
                      "note": "T2D + T1D + Fst, back-to-back runs of one plan on one stream"},
           "pipeline_bytes_note": "SURVEY 8(d): 12 B/SNP + 64 B/window per pass over the time per pass; "
                                  "pipeline_*: independent passes overlapped on 2 HIP streams as in the bench's "
                                  "own loop (the 'overlapped' entry, T2D + T1D + Fst)",
           "windows": nwin,
           "workload": "config 3 stream on 1 GPU: 32 chrom x 1.5625e6 SNPs, 20 kb, per-chromosome bg, T2D + T1D + Fst"}
    pl.close()
    # independent passes overlapped on 2 HIP streams (the bench's own mode), the scan kernel capped at one
    # workgroup per CU so that the next pass's bandwidth-bound k_prep runs beside the previous pass's
    # compute-bound scan (profiles/r03h_streams_wgs.txt): with Fst (the metric's statistics) and without
    # (T2D + T1D, the reference's statistics)
    import torch
    from sfs2d.engine import Plan
    streams = [torch.cuda.current_stream().cuda_stream, torch.cuda.Stream().cuda_stream]
    for key, fst in (("overlapped", True), ("t2d_t1d_overlapped", False)):
        cfg2 = ScanConfig(n1p=POP, n2p=POP, window=WS, fst=fst, scan_wgs_per_cu=1)
        plans = [eng.plan(dev, cfg2) for _ in range(2)]
        outs = [torch.zeros((plans[0].nrec, 64), dtype=torch.uint8, device="cuda") for _ in range(2)]
        ptrs = [o.data_ptr() for o in outs]
        Plan.run_streams(plans, streams, 8, ptrs)
        torch.cuda.synchronize()
        reps = []   # three repetitions, the median reported (the box's host and neighbours make single runs noisy)
        for _ in range(3):
            t0 = time.perf_counter()
            Plan.run_streams(plans, streams, 8 * steps, ptrs)
            torch.cuda.synchronize()
            reps.append((time.perf_counter() - t0) / (8 * steps))
        wo = sorted(reps)[1]
        for q in plans:
            q.check()
        if not torch.equal(outs[0], outs[1]):
            raise RuntimeError("config-3 overlapped passes disagree")
        if fst and not np.array_equal(plans[0].read_fst(), plans[1].read_fst(), equal_nan=True):
            raise RuntimeError("config-3 overlapped passes disagree (Fst)")
        out[key] = {
            "pipeline_GBs": bp / wo / 1e9, "pipeline_frac": bp / wo / 1e9 / HBM_PEAK_GBS, "pipeline_ms": wo * 1e3,
            "pipeline_ms_reps": [r * 1e3 for r in reps], "windows_per_s": nwin / wo,
            "note": ("T2D + T1D + Fst" if fst else "T2D + T1D only (the reference's statistics; Hudson Fst not computed)")
                    + ": 2 plans on 2 HIP streams, passes overlapped, scan kernel capped at 1 workgroup per CU; "
                      "SURVEY 8(d) bytes over the time per pass"}
        for q in plans:
            q.close()
    dev.close()
    o = out["overlapped"]
    out.update({"pipeline_GBs": o["pipeline_GBs"], "pipeline_frac": o["pipeline_frac"], "pipeline_ms": o["pipeline_ms"],
                "windows_per_s": o["windows_per_s"]})
    return out


def launch_ranks(n):
    """``--gpus N`` with no launcher around this process: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1) before this process
    imports torch or touches the GPU, wait for them, and return the first failing status (the other
    ranks are then killed by PID)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for q in list(live):
            c = q.poll()
            if c is None:
                continue
            live.remove(q)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 1
                for o in live:
                    o.kill()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hbm-stream", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the VCF -> CSV end-to-end timing")
    ap.add_argument("--streams", type=int, default=3,
                    help="consecutive steps round-robin over this many plans, each on its own HIP stream "
                         "(independent passes overlap; sfs2d_plan_run_streams)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    # hardware queues per process: HIP maps streams onto GPU_MAX_HW_QUEUES queues (4 on the box); S
    # pass streams + the library's and torch's own need more than 4 or two passes share a queue and
    # serialise (3 streams: 1.35e8 windows/s with 4 queues, 1.92-1.94e8 with 6-8; profiles/r02h_*).
    # Set before the HIP runtime starts (torch imported below; rank processes inherit it).
    need = max(1, args.streams) + 4
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < need:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(8, need)))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} launched with WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    ndev = torch.cuda.device_count()
    if ndev < world or local >= ndev:
        raise RuntimeError(f"bench.py --gpus {world}: rank {rank} needs device {local}, {ndev} visible")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("nccl", rank=rank, world_size=world)
        world = dist.get_world_size()   # n_gpus from the communicator

    from sfs2d import _lib as L
    from sfs2d.engine import Engine, Plan, ScanConfig
    from sfs2d.synth import synth_genome

    # weak scaling: every rank scans its own chromosome (seed 12345 + rank) -- whole chromosomes are
    # the shard unit of per-chromosome-background scans
    p = synth_genome(1, N_SNP, POP, POP, seed=12345 + rank)
    eng = Engine.get(local)
    scan_s = torch.cuda.Stream(device=local)    # the HIP library's stream (and the final gather's)
    torch.cuda.set_stream(scan_s)
    eng.set_stream(scan_s.cuda_stream)
    dev = eng.upload(p)
    cfg = ScanConfig(n1p=POP, n2p=POP, window=WS, fst=True)
    ns = max(1, args.streams)
    plans = [eng.plan(dev, cfg) for _ in range(ns)]
    pl = plans[0]
    nrec = pl.nrec
    cdev = f"cuda:{local}"
    rows = nrec
    if world > 1:   # shards differ in window count: tables are padded to the largest (rows flagged empty)
        c = torch.tensor([nrec], dtype=torch.int64, device=cdev)
        dist.all_reduce(c, op=dist.ReduceOp.MAX)
        rows = int(c.item())
    sstreams = [scan_s.cuda_stream] + [torch.cuda.Stream(device=local).cuda_stream for _ in range(ns - 1)]
    ev_done = [torch.cuda.Event() for _ in range(ns)]
    outs = [torch.zeros((rows, 64), dtype=torch.uint8, device=cdev) for _ in range(ns)]
    for o in outs:
        o[nrec:, 39] = 0x80   # padding rows: flags = SFS2D_W_EMPTY
    optrs = [o.data_ptr() for o in outs]
    gathered = torch.empty((world * rows, 64), dtype=torch.uint8, device=cdev) if world > 1 else None
    last = (args.steps - 1) % ns   # the table the last timed step writes

    def gather_final(k):
        # the single collective: every rank's final window table to every rank (RCCL over xGMI),
        # ordered after the scans of all the plans' streams
        for j, e in enumerate(ev_done):
            e.record(torch.cuda.ExternalStream(sstreams[j]))
            scan_s.wait_event(e)
        dist.all_gather_into_tensor(gathered, outs[k])

    pl.run(optrs[0])
    pl.check()
    # warmup: the same loop, and (N > 1) the collective once (RCCL communicators are made lazily)
    Plan.run_streams(plans, sstreams, args.warmup * ns, optrs)
    if world > 1:
        gather_final(last)
    torch.cuda.synchronize()
    # HIP events around the scan kernel (the roofline's) and k_bg_slice of sampled timed runs of plan 0,
    # carried in their dispatch packets on the stream the kernels run on (events around all three
    # kernels of every 8th run cost ~2 us per step, around these two ~1 us: tools/timing_overhead.py);
    # k_prep is timed in an untimed pass after the timed loop.  Short runs (the driver's 20 steps)
    # sample every 2nd run of plan 0 so that the average is over >= 5 launches.
    every = 8 if args.steps >= 160 else 2
    pl.set_timing(args.steps, every=every, kernels=6)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # the timed loop, the same at every N: step i = one scan pass of plan i % ns on stream i % ns;
    # with N > 1 ranks, then one gather of the final window tables
    Plan.run_streams(plans, sstreams, args.steps, optrs)
    if world > 1:
        gather_final(last)
    t_enq = time.perf_counter() - t0   # host time to enqueue the timed steps (diagnostic)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    nr, (_, k2, k3) = pl.timing_read()
    pl.set_timing(16, every=1)   # k_prep (and the other two again), one stream, outside the timed region
    pl.run_many(16, optrs[0])
    _, (k1, _, k3_untimed) = pl.timing_read()
    pl.set_timing(0)
    for k, q in enumerate(plans):   # every plan's last pass wrote the same records (independent state)
        q.check()
        if not torch.equal(outs[k][:nrec], outs[0][:nrec]):
            raise RuntimeError(f"plan {k} on stream {k} disagrees with plan 0")
    recs = np.frombuffer(outs[0][:nrec].cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
    nwin_rank = int(((recs["flags"] & L.W_EMPTY) == 0).sum())
    total_windows = nwin_rank
    if world > 1:
        g = gathered.view(world, rows, 64)
        if not torch.equal(g[rank][:nrec], outs[0][:nrec]):
            raise RuntimeError("the gathered table disagrees with this rank's own")
        allr = np.frombuffer(g.cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
        total_windows = int(((allr["flags"] & L.W_EMPTY) == 0).sum())
    value = total_windows * args.steps / dt

    if rank == 0:
        b3 = algorithmic_bytes(p.n, nrec, nwin_rank, "k3")
        # the roofline's duration: with overlapped passes (ns > 1) a kernel's event interval in the
        # timed region also holds the time its workgroups wait for CUs that the other passes' kernels
        # occupy (k_scan_w 14-16 us there vs 9.5-9.8 us in rocprofv3's kernel trace of the same
        # command), so the kernel's own duration comes from the single-stream pass of 16 runs after
        # the timed loop (the same kernel, data and dispatch-packet events)
        k3_roof = k3_untimed if ns > 1 else k3
        achieved = b3 / (k3_roof * 1e-3) / 1e9
        bp = algorithmic_bytes(p.n, nrec, nwin_rank, "pipeline") * world
        step_s = dt / args.steps
        traffic, tsrc = pmc_traffic("k_scan_w", pl.grids()[1])
        line = {
            "metric": "genomic windows/s (T2D+T1D+Fst) at 20 kb, n1=n2=50; HBM GB/s fraction",
            "value": value, "unit": "windows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3, "host_enqueue_ms_per_step": t_enq / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (SURVEY 8d generator, seed 12345+rank)",
            "config": {"workload": "configs[1]: synthetic 1 chromosome x 1e6 SNPs per GPU, 20 kb windows, "
                                   "n1=n2=50 haploid (pop_size 25/25), per-chromosome background",
                       "snps_per_gpu": p.n, "windows_per_gpu": nwin_rank, "windows_all_gpus": total_windows,
                       "window_bp": WS,
                       "stats": "T2D, T1D_p1, T1D_p2 (reference semantics) + Hudson Fst (DESIGN.md; not in the "
                                "reference, parity vs its own oracle restatement)",
                       "parallelism": f"one chromosome per GPU ({world} GPU(s)), no data-path collective; "
                                      f"{ns} plans on {ns} HIP streams, steps round-robin (passes overlap)"
                                      + ("; one RCCL all-gather of the final window tables in the timed region"
                                         if world > 1 else "")},
            "kernels_ms": {"k_prep": k1, "k_bg_slice": k2, "k_scan_w": k3, "k_scan_w_untimed_pass": k3_untimed,
                           "timed_runs_sampled": nr, "exact_path_windows": pl.stats(),
                           "note": f"k_bg_slice / k_scan_w: events in every {every}th timed run of plan 0; k_prep: 16 "
                                   "runs after the timed loop (one stream, untimed)"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "k_scan_w", "ms": k3_roof, "ms_timed_region": k3, "algorithmic_bytes": b3,
                         "note": "k_scan_w: algorithmic bytes 4 B/SNP + 96 B/slot per launch over its average "
                                 + (f"duration in the single-stream pass of 16 runs after the timed loop (kernel "
                                    "start/end events in the dispatch packets; in the timed region, every "
                                    f"{every}th run of plan 0, the interval also holds the wait for CUs held by "
                                    "the other streams' passes: ms_timed_region); " if ns > 1 else
                                    f"duration (kernel start/end events in the dispatch packets of every {every}th "
                                    "timed run); ")
                                 + "the 8 MB config-2 stream is MALL-resident (see roofline_hbm for the HBM-sized "
                                 "stream); traffic: " + (tsrc or "no PMC pass committed")},
            "roofline_pipeline": {"bound": "hbm", "achieved": bp / step_s / 1e9, "peak": HBM_PEAK_GBS * world,
                                  "unit": "GB/s", "frac": bp / step_s / 1e9 / (HBM_PEAK_GBS * world),
                                  "note": "whole step over all GPUs (SURVEY 8(d): 12 B/SNP + 64 B/window) over "
                                          "ms_per_step"},
        }
        if not args.no_hbm_stream and world == 1:
            line["roofline_hbm"] = hbm_stream_roofline(eng)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(p)
        if not args.no_e2e and world == 1:
            line["end_to_end_vcf_csv"] = end_to_end()
        print(json.dumps(line), flush=True)
    for q in plans[::-1]:
        q.close()
    dev.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
