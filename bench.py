#!/usr/bin/env python3
"""Benchmark: genomic windows/s of the 2D-SFS composite-likelihood scan (BASELINE.json metric).

Headline (``value``): BASELINE configs[2] -- the synthetic whole genome, 32 chromosomes x 1.5625e6 =
5e7 SNPs (SURVEY 8d generator, seed 777), n1 = n2 = 50 haploid (pop_size 25/25), 20 kb fixed-bp
windows, every chromosome its own background (combined_scan semantics), T2D + T1D_p1 + T1D_p2 +
Hudson Fst -- SHARDED BY WINDOW over the N GPUs (strong scaling: the same genome at every N).  Rank
r holds the SNPs [c_r, c_r+1) of sfs2d.dist.split_points (cuts at window starts nearest k n / N; at
N | 32 they are chromosome ends, so no chromosome's background spans two ranks).  A step = one full
scan pass over the genome: on every rank, background histograms + window segmentation (k_prep),
then the window scan (k_scan_w, its table prologue fused) -> HBM-resident 64-B window records + Fst.
Consecutive passes are independent: they go round-robin over 2 plans on 2 HIP streams (the scan
capped at one workgroup per CU so the next pass's bandwidth-bound k_prep finds CUs beside it).  At
N > 1 EVERY pass's window table (64-B records + 8-B Fst per slot) is all-gathered to every rank over
RCCL / xGMI inside the timed region (run_loop_gathered: groups of passes, each group's gather
overlapped with the next group's passes), as each reference scan returns its whole per-window dict;
`value` counts gathered windows only.  At N = 1 the 5e7-SNP stream (~609 MB per pass) is far past
the 256 MB Infinity Cache: the HBM roofline is measured on it.

Second key ``config2_weak``: BASELINE configs[1] (one 1e6-SNP chromosome per GPU, weak scaling, 3 plans
on 3 streams), the round-1..3 headline, with its own roofline and the single-stream pass latency.
``config4_sims`` / ``config5_snp_windows`` (N = 1): BASELINE configs[3] (sims_scan at full size: 4 x
2,500 replicates generated in HBM, 101 x 101 grid) and configs[4] (500-SNP windows, 201 x 151 grid),
each with the roofline of its scan kernel (k_scan_gw).

`--gpus N` with no launcher: this script starts the N rank processes itself (before touching the
GPU) and exits with their status; under torchrun, WORLD_SIZE must equal N, and a box with fewer
than N GPUs fails instead of reporting fewer.

Each loop runs untimed passes for SETTLE_S of wall time before its W warmup steps (the GPU's clock
ramp out of idle: a 100-step config-3 loop is ~20 ms), then times exactly K steps.

Prints ONE JSON line on rank 0.  ``roofline``: the dominant kernel (k_scan_w) of the headline workload,
algorithmic bytes per launch over its average duration in the timed steps (HIP start / end events in
its dispatch packets, >= 10 of the timed passes, on the stream it runs on; its one-stream duration is
rank0.scan_alone_ms).  ``cpu_baseline``: the C oracle (the reference's dense per-window algorithm,
OpenMP) on the box's host cores over a bounded sample of the same genome (its first chromosome).
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
SETTLE_S = 0.3          # untimed passes before each loop's warmup (the GPU's clock ramp; run_loop)
POP = 25
WS = 20000
C3_NCHROM, C3_PER, C3_SEED = 32, 1_562_500, 777
C2_SNP, C2_SEED = 1_000_000, 12345
METRIC = "genomic windows/s (T2D+T1D+Fst) at 20 kb, n1=n2=50; HBM GB/s fraction"


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
        if r.get("kernel", "").startswith(kernel + "<") and int(r.get("grid", -1)) == int(grid):
            return r["read_bytes"] + r["write_bytes"], d.get("source", path)
    return None, None


def cpu_baseline(p):
    """The CPU baseline on this box's host cores: the C restatement of the oracle (oracle/sfs_oracle_c.c,
    the reference's dense per-window algorithm, OpenMP over windows; test infrastructure, pinned to
    the numpy oracle) over a bounded sample of the headline genome (its first chromosome), repeated
    for >= 3 s; beside it the numpy oracle itself (dense grids + scipy multinomial.logpmf, as the
    reference computes them) on one core over the same sample."""
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
    q = p.subset_chroms([0])
    q = type(q)(q.counts[:200_000], q.pos[:200_000], np.array([0, 200_000]), q.chrom_names, q.ann_id[:200_000],
                q.ann_names, q.pop1, q.pop2)
    cfg = O.Cfg(POP, POP)
    t1 = time.perf_counter()
    res = O.combined_scan(q, WS, cfg)
    dt1 = time.perf_counter() - t1
    return {"value": nwin * reps / dt, "unit": "windows/s", "cores": threads, "kind": "port",
            "sample": f"chromosome 0 of the headline genome ({p.n} SNPs, {nwin} windows) x {reps} in {dt:.1f} s: "
                      "oracle/sfs_oracle_c.c (the reference's dense per-window grids and scipy's logpmf "
                      f"closed form, numpy's pairwise p-sums; T2D + T1D, no Fst), OpenMP over windows on "
                      f"{threads} host threads",
            "numpy_oracle_1core": {"value": len(res) / dt1, "unit": "windows/s", "cores": 1,
                                   "sample": f"oracle/sfs_oracle.combined_scan on its first {q.n} SNPs ({dt1:.1f} s)"}}


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


SHARED_GPU = os.environ.get("SFS2D_BENCH_SHARED_GPU") == "1"


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


class Ctx:
    """What both workloads share on a rank: the process group, the engine and the library's stream."""

    def __init__(self, world, rank, local, nstreams=3):
        import torch
        import torch.distributed as dist
        from sfs2d.engine import Engine
        self.torch, self.dist = torch, dist
        self.world, self.rank, self.local = world, rank, local
        self.shared = SHARED_GPU and world > 1   # rehearsal: all ranks on GPU 0, gloo (see main)
        self.cdev = f"cuda:{local}"
        self.eng = Engine.get(local)
        self.scan_s = torch.cuda.Stream(device=local)   # the HIP library's stream (and the final gather's)
        torch.cuda.set_stream(self.scan_s)
        self.eng.set_stream(self.scan_s.cuda_stream)
        # the passes' streams, created once for every loop of the run: HIP maps streams onto the
        # process's few hardware queues (4) in creation order, and a loop whose streams came after the
        # earlier loops' shared queues (serialised passes: config 2 at 38 us per pass instead of 13)
        self.streams = [self.scan_s.cuda_stream] + [torch.cuda.Stream(device=local).cuda_stream
                                                    for _ in range(max(2, nstreams) - 1)]

    def max_over_ranks(self, x, dtype=None):
        if self.world == 1:
            return x
        torch = self.torch
        t = torch.tensor([x], dtype=dtype or (torch.float64 if isinstance(x, float) else torch.int64),
                         device="cpu" if self.shared else self.cdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return t.item()


def sample_every(passes_per_plan):
    """Every how many passes (per plan) a timed loop's kernels carry start / end events: 2 sampled passes
    per plan, the first and the last one (a perturbed last pass shifts no later pass).  The events perturb the two streams' overlap: at 20 steps,
    sampling every 2nd pass per plan put 1-2 of 8 runs of the driver's command into the slow phase
    (0.19-0.22 ms), every pass 4 of 8, every 10th none (0.180-0.183 ms, profiles/r06ac_*).
    SFS2D_BENCH_EVERY overrides."""
    ev = os.environ.get("SFS2D_BENCH_EVERY")
    return int(ev) if ev else max(1, passes_per_plan - 1)


def run_loop(cx, plans, steps, warmup, label, time_kernels=False, graph_runs=0):
    """The timed loop shared by both workloads: `warmup` untimed rounds, then exactly `steps` passes
    round-robin over the plans (plan i % S on stream i % S), then (N > 1) ONE all-gather of every
    rank's final window table; barrier + synchronize on both sides, the max over ranks.  Returns the
    wall time, the device time of the passes and of the gather (HIP events on the gather's stream),
    the host enqueue time, the gathered table (host) and this rank's final table."""
    torch, dist = cx.torch, cx.dist
    from sfs2d.engine import Plan
    ns = len(plans)
    nrec = plans[0].nrec
    rows = int(cx.max_over_ranks(nrec))   # tables padded to the largest shard (rows flagged empty)
    if ns > len(cx.streams):
        raise ValueError(f"{label}: {ns} plans, {len(cx.streams)} streams")
    sstreams = cx.streams[:ns]
    outs = [torch.zeros((rows, 64), dtype=torch.uint8, device=cx.cdev) for _ in range(ns)]
    for o in outs:
        o[nrec:, 39] = 0x80   # padding rows: flags = SFS2D_W_EMPTY
    optrs = [o.data_ptr() for o in outs]
    gathered = torch.empty((cx.world * rows, 64), dtype=torch.uint8, device=cx.cdev) if cx.world > 1 else None
    ev_done = [torch.cuda.Event() for _ in range(ns)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    last = (steps - 1) % ns   # the table the last timed step writes

    def gather_final(k, timed):
        # the single collective: every rank's final window table to every rank (RCCL over xGMI),
        # ordered after the passes of all the plans' streams
        for j, e in enumerate(ev_done):
            e.record(torch.cuda.ExternalStream(sstreams[j]))
            cx.scan_s.wait_event(e)
        if timed:
            ev[1].record(cx.scan_s)
        if cx.world > 1 and cx.shared:
            # SFS2D_BENCH_SHARED_GPU (a rehearsal of N > 1 with every rank on one GPU, gloo): host-staged
            parts = [torch.empty_like(outs[k], device="cpu") for _ in range(cx.world)]
            dist.all_gather(parts, outs[k].cpu())
            gathered.copy_(torch.cat(parts).to(cx.cdev))
        elif cx.world > 1:
            dist.all_gather_into_tensor(gathered, outs[k])
        if timed:
            ev[2].record(cx.scan_s)

    plans[0].run(optrs[0])
    plans[0].check()
    # graph_runs > 0: the run sequence captured once into a HIP graph of graph_runs runs (Plan.graph),
    # replayed steps / graph_runs times -- one host launch per replay instead of three per run
    rg = None
    if graph_runs:
        if steps % graph_runs or time_kernels:
            raise ValueError(f"{label}: graph of {graph_runs} runs, {steps} steps (timing: {time_kernels})")
        rg = Plan.graph(plans, sstreams, graph_runs, optrs)

    def enqueue(n):
        if rg is not None:
            rg.launch(-(-n // graph_runs))
            return -(-n // graph_runs) * graph_runs
        Plan.run_streams(plans, sstreams, n, optrs)
        return n

    every = sample_every(-(-steps // len(plans)))
    if time_kernels:   # the timing events made now: re-armed right before the timed steps at no cost
        for q in plans:
            q.set_timing(steps, every=every, kernels=5)
            q.set_timing(0)
    # device settle (untimed): passes for SETTLE_S of wall time before the warmup, so that the timed
    # steps run at the GPU's sustained clock rather than on its ramp out of idle (a 100-step timed loop
    # is ~20 ms: measured 0.195 ms per step after 10 warmup passes, 0.181 after 600)
    t_s = time.perf_counter()
    settle = 0
    while time.perf_counter() - t_s < SETTLE_S:
        settle += enqueue(8 * ns)
        torch.cuda.synchronize()
    enqueue(warmup * ns)
    gather_final(last, False)
    torch.cuda.synchronize()
    if cx.world > 1:
        dist.barrier()
    # k_prep / scan-kernel durations over the timed steps themselves (start / end events in the
    # kernels' dispatch packets of 2 timed passes per plan, sample_every): the overlapped launches the
    # roofline prices
    if time_kernels:
        for q in plans:
            q.set_timing(steps, every=every, kernels=5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev[0].record(cx.scan_s)
    enqueue(steps)
    gather_final(last, True)
    t_enq = time.perf_counter() - t0   # host time to enqueue the timed steps (diagnostic)
    torch.cuda.synchronize()
    if cx.world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kt = [q.timing_read() for q in plans] if time_kernels else []
    if time_kernels:
        for q in plans:
            q.set_timing(0)
    nk = sum(n for n, _ in kt)
    k_timed = (sum(n * k[0] for n, k in kt) / max(1, nk), sum(n * k[2] for n, k in kt) / max(1, nk))
    dt = float(cx.max_over_ranks(dt))
    dev_ms = float(cx.max_over_ranks(float(ev[0].elapsed_time(ev[1]))))
    gat_ms = float(cx.max_over_ranks(float(ev[1].elapsed_time(ev[2]))))
    for k, q in enumerate(plans):   # every plan's last pass wrote the same records (independent state)
        q.check()
        if not torch.equal(outs[k][:nrec], outs[0][:nrec]):
            raise RuntimeError(f"{label}: plan {k} on stream {k} disagrees with plan 0")
    mine = outs[last][:nrec].cpu().numpy()
    if cx.world > 1:
        g = gathered.view(cx.world, rows, 64)
        if not torch.equal(g[cx.rank][:nrec], outs[last][:nrec]):
            raise RuntimeError(f"{label}: the gathered table disagrees with this rank's own")
        allr = g.cpu().numpy().reshape(-1, 64)
    else:
        allr = mine
    if rg is not None:
        rg.close()
    return {"dt": dt, "device_ms": dev_ms, "gather_ms": gat_ms, "t_enq": t_enq, "rows": rows,
            "gathered": allr, "mine": mine, "streams": ns, "settle_passes": settle,
            "k_timed_ms": k_timed, "k_timed_samples": nk}


def run_loop_gathered(cx, plans, steps, warmup, label, nstreams=2, time_kernels=False):
    """The N > 1 timed loop: every pass's window table (64-B records + the 8-B Fst column) is
    all-gathered to every rank, as each reference scan returns its whole per-window dict
    (twoDSFS_class.py:882-891).  Passes go in groups of P = len(plans) (plan j on stream j % nstreams, one
    sfs2d_plan_run_streams call per group), each pass writing into its own slice of the group's buffer;
    the group's buffer is then all-gathered (RCCL over xGMI) on a separate stream while the next group's
    passes run, into one of NB = 2 buffer slots (a slot is reused only after its gather finished).  The
    timed region is exactly `steps` passes and their `steps` gathered tables (a last partial group when
    P does not divide steps); barrier + synchronize on both sides, max over ranks."""
    torch, dist = cx.torch, cx.dist
    from sfs2d.engine import Plan
    P = len(plans)
    nrec = plans[0].nrec
    rows = int(cx.max_over_ranks(nrec))   # tables padded to the largest shard (rows flagged empty)
    fst = plans[0].cfg.fst
    if nstreams > len(cx.streams):
        raise ValueError(f"{label}: {nstreams} streams, {len(cx.streams)} available")
    sstreams = [cx.streams[j % nstreams] for j in range(P)]
    used = cx.streams[:nstreams]
    NB = 2
    rec_b, fst_b = rows * 64, (rows * 8 if fst else 0)
    per = P * (rec_b + fst_b)   # bytes of one group's tables on one rank
    bufs = [torch.zeros(per, dtype=torch.uint8, device=cx.cdev) for _ in range(NB)]
    for b in bufs:
        v = b[: P * rec_b].view(P, rows, 64)
        v[:, nrec:, 39] = 0x80   # padding rows: flags = SFS2D_W_EMPTY
    gathered = [torch.empty(cx.world * per, dtype=torch.uint8, device=cx.cdev) for _ in range(NB)]
    gs = torch.cuda.Stream(device=cx.local)   # the gathers' stream
    ev_pass = [torch.cuda.Event() for _ in range(nstreams)]
    ev_gdone = [torch.cuda.Event() for _ in range(NB)]
    ev_g = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    gath_groups = [0]
    tev = []   # (start, end) events around each timed group's all-gather

    def group(g, npass, timed):
        slot = g % NB
        if g >= NB:   # the slot's previous gather has read it
            for s in used:
                torch.cuda.ExternalStream(s).wait_event(ev_gdone[slot])
        base = bufs[slot].data_ptr()
        if fst:
            for j in range(npass):
                plans[j].set_fst_out(base + P * rec_b + j * fst_b)
        Plan.run_streams(plans[:npass], sstreams[:npass], npass, [base + j * rec_b for j in range(npass)])
        for k, s in enumerate(used[: min(nstreams, npass)]):
            ev_pass[k].record(torch.cuda.ExternalStream(s))
            gs.wait_event(ev_pass[k])
        with torch.cuda.stream(gs):
            if timed:
                tev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                tev[-1][0].record(gs)
            if cx.shared:   # SFS2D_BENCH_SHARED_GPU rehearsal (gloo, host-staged)
                parts = [torch.empty(per, dtype=torch.uint8) for _ in range(cx.world)]
                dist.all_gather(parts, bufs[slot].cpu())
                gathered[slot].copy_(torch.cat(parts).to(cx.cdev))
            else:
                dist.all_gather_into_tensor(gathered[slot], bufs[slot])
            if timed:
                tev[-1][1].record(gs)
            ev_gdone[slot].record(gs)
        gath_groups[0] += 1

    def passes(n, timed, g0=0):
        g = g0
        while n > 0:
            k = min(P, n)
            group(g, k, timed)
            n -= k
            g += 1
        return g

    g = passes(P, False)
    torch.cuda.synchronize()
    for q in plans:
        q.check()
    every = sample_every(-(-steps // len(plans)))
    if time_kernels:   # the timing events made now: re-armed right before the timed steps at no cost
        for q in plans:
            q.set_timing(steps, every=every, kernels=5)
            q.set_timing(0)
    t_s = time.perf_counter()
    settle = 0
    while time.perf_counter() - t_s < SETTLE_S:
        g = passes(8 * P, False, g)
        torch.cuda.synchronize()
        settle += 8 * P
    g = passes(warmup * nstreams, False, g)
    torch.cuda.synchronize()
    dist.barrier()
    if time_kernels:
        for q in plans:
            q.set_timing(steps, every=every, kernels=5)
    torch.cuda.synchronize()
    g0 = g
    t0 = time.perf_counter()
    ev_g[0].record(gs)
    g = passes(steps, True, g)
    ev_g[1].record(gs)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    kt = [q.timing_read() for q in plans] if time_kernels else []
    if time_kernels:
        for q in plans:
            q.set_timing(0)
    nk = sum(n for n, _ in kt)
    k_timed = (sum(n * k[0] for n, k in kt) / max(1, nk), sum(n * k[2] for n, k in kt) / max(1, nk))
    dt = float(cx.max_over_ranks(dt))
    span_ms = float(cx.max_over_ranks(float(ev_g[0].elapsed_time(ev_g[1]))))
    gat_ms = float(cx.max_over_ranks(float(sum(a.elapsed_time(b) for a, b in tev))))
    # every gathered table of the last groups: this rank's section equals its own pass output, every plan's
    # table the same (independent passes over the same shard), and the windows of all ranks counted
    last_groups = sorted({(g - 1 - i) for i in range(min(NB, g - g0))})
    nwin_pass = None
    for gg in last_groups:
        slot = gg % NB
        npass = P if (gg < g - 1 or steps % P == 0) else steps % P
        G = gathered[slot].view(cx.world, per)
        for q in plans:
            q.check()
        own = bufs[slot][: npass * rec_b].view(npass, rows, 64)
        for j in range(npass):
            if not torch.equal(own[j][:nrec], own[0][:nrec]):
                raise RuntimeError(f"{label}: pass {j} of group {gg} disagrees with pass 0")
        if not torch.equal(G[cx.rank], bufs[slot]):
            raise RuntimeError(f"{label}: the gathered tables disagree with this rank's own")
        tabs = G[:, : P * rec_b].reshape(cx.world, P, rows, 64)[:, :npass].cpu().numpy()
        counts = {n_windows(tabs[:, j].reshape(-1, 64)) for j in range(npass)}
        if len(counts) != 1:
            raise RuntimeError(f"{label}: gathered tables hold different window counts {counts}")
        nwin_pass = counts.pop()
    if fst:
        for q in plans:
            q.set_fst_out(None)
    mine = bufs[(g - 1) % NB][:rec_b].view(rows, 64)[:nrec].cpu().numpy()
    allr = gathered[(g - 1) % NB].view(cx.world, per)[:, :rec_b].reshape(-1, 64).cpu().numpy()
    return {"dt": dt, "device_ms": span_ms, "gather_ms": gat_ms, "t_enq": t_enq, "rows": rows,
            "gathered": allr, "mine": mine, "streams": nstreams, "settle_passes": settle,
            "k_timed_ms": k_timed, "k_timed_samples": nk, "windows_per_pass_gathered": nwin_pass,
            "gathers": g - g0, "group": P, "gathered_bytes_per_pass": cx.world * (rec_b + fst_b)}


def kernel_times(plan, runs=16):
    """k_prep / k_bg_slice / scan kernel durations (events in their dispatch packets), one stream, untimed."""
    plan.set_timing(runs, every=1)
    plan.run_many(runs)
    _, (k1, k2, k3) = plan.timing_read()
    plan.set_timing(0)
    plan.check()
    return k1, k2, k3


def dense_kernel_samples(cx, plans, loops, steps):
    """Untimed, after the timed loop: `loops` more loops of `steps` passes over the same plans and
    streams, each started and sampled as the timed loop is (staggered start, synchronised at its end,
    kernel events on each plan's first and last pass, sample_every) -- the timed loop's condition
    repeated, so that the overlapped k_prep / scan durations rest on 2 x plans x loops launches instead of
    2 x plans.  (One long unsynchronised loop drifts between the streams' two phases, and events on every
    pass put it in the slow one: 0.19-0.26 / 0.275 ms per scan launch, profiles/r06ah, r06ai.)
    Returns (k_prep ms, scan ms, launches sampled)."""
    from sfs2d.engine import Plan
    ns = len(plans)
    every = sample_every(-(-steps // ns))
    acc = [0, 0.0, 0.0]
    for _ in range(loops):
        for q in plans:
            q.set_timing(steps, every=every, kernels=5)
        Plan.run_streams(plans, cx.streams[:ns], steps)
        cx.torch.cuda.synchronize()
        for q in plans:
            n, k = q.timing_read()
            acc[0] += n
            acc[1] += n * k[0]
            acc[2] += n * k[2]
    for q in plans:
        q.set_timing(0)
        q.check()
    nk = max(1, acc[0])
    return (acc[1] / nk, acc[2] / nk, acc[0])


def single_pass_ms(cx, plan, runs=10):
    """One plan back to back on one stream: the latency of a single pass (no overlap)."""
    torch = cx.torch
    plan.run_many(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    plan.run_many(runs)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / runs * 1e3


def n_windows(table):
    from sfs2d import _lib as L
    r = np.frombuffer(np.ascontiguousarray(table).tobytes(), dtype=L.WINDOW_DTYPE)
    return int(((r["flags"] & L.W_EMPTY) == 0).sum())


def config3_cuts(p, cfg, world):
    """Rank r scans SNPs [cuts[r], cuts[r+1]): sfs2d.dist.split_points (window starts nearest k n / N);
    when one of them falls inside a chromosome (N not dividing 32), whole-chromosome shards instead
    (sfs2d.dist.shard_chromosomes), so that no background spans two ranks inside the timed loop."""
    from sfs2d import dist as D
    cuts = D.split_points(p, cfg, world)
    ends = set(p.chrom_off.tolist())
    if not all(c in ends for c in cuts):
        sh = D.shard_chromosomes(p.chrom_off, world)
        cuts = [int(p.chrom_off[a]) for a, _ in sh] + [p.n]
    return cuts


def config3_strong(cx, args):
    """The headline: config 3, sharded by window over the ranks, strong scaling."""
    from sfs2d import dist as D
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(C3_NCHROM, C3_PER, POP, POP, seed=C3_SEED)
    cfg = ScanConfig(n1p=POP, n2p=POP, window=WS, fst=True, scan_wgs_per_cu=1)
    cuts = config3_cuts(p, cfg, cx.world)
    sub, c0 = p.slice_snps(cuts[cx.rank], cuts[cx.rank + 1])
    dev = cx.eng.upload(sub)
    ns = 2
    if cx.world > 1:
        # every pass's table gathered (run_loop_gathered): groups of P passes on the 2 streams, P | steps
        P = next(k for k in (args.group, 4, 2, 1) if k >= 1 and args.steps % k == 0)
        plans = [cx.eng.plan(dev, cfg) for _ in range(max(P, ns))]
        r = run_loop_gathered(cx, plans[:P] if P >= ns else plans, args.steps, args.warmup, "config 3",
                              nstreams=ns, time_kernels=True)
        total_windows = r["windows_per_pass_gathered"]
    else:
        plans = [cx.eng.plan(dev, cfg) for _ in range(ns)]
        r = run_loop(cx, plans, args.steps, args.warmup, "config 3", time_kernels=True)
        total_windows = n_windows(r["gathered"])
    win_rank = n_windows(r["mine"])
    k1, _, k3 = kernel_times(plans[0])
    dense = dense_kernel_samples(cx, plans, 10, args.steps) if cx.rank == 0 else None
    # a single scan of the genome as a user runs it: the default plan (no scan grid cap), back to back
    # on one stream
    one = None
    if cx.rank == 0:
        solo = cx.eng.plan(dev, ScanConfig(n1p=POP, n2p=POP, window=WS, fst=True))
        one = single_pass_ms(cx, solo, runs=50)
        solo.close()
    extra = {}
    if cx.world == 1 and not args.no_variants:
        # what Hudson's Fst costs the pass: the same loop without Fst (the reference's statistics) and
        # with it, interleaved three times each (box-to-box clock drift moves both alike); medians
        cfg2 = ScanConfig(n1p=POP, n2p=POP, window=WS, fst=False, scan_wgs_per_cu=1)
        q = [cx.eng.plan(dev, cfg2) for _ in range(ns)]
        ms_f, ms_n = [], []
        for _ in range(3):
            rr = run_loop(cx, q, args.steps, args.warmup, "config 3 without Fst")
            ms_n.append(rr["dt"] / args.steps * 1e3)
            rf = run_loop(cx, plans, args.steps, args.warmup, "config 3 (Fst, repeat)")
            ms_f.append(rf["dt"] / args.steps * 1e3)
        for x in q:
            x.close()
        mf, mn = float(np.median(ms_f)), float(np.median(ms_n))
        extra["t2d_t1d_only"] = {"ms_per_step": mn, "windows_per_s": n_windows(rr["gathered"]) / (mn * 1e-3),
                                 "ms_per_step_runs": ms_n, "with_fst_ms_per_step_runs": ms_f,
                                 "note": "the same loop, T2D + T1D only (Hudson Fst not computed); three loops "
                                         "interleaved with three more of the Fst loop, medians"}
        extra["fst_cost_interleaved"] = mf / mn - 1.0
        # BASELINE configs[2] names 20 kb AND 500 kb windows: both from one k_prep pass (sfs2d_plan_attach:
        # the 500 kb plan scanned from the 20 kb base's pass), T2D + T1D + Fst on both
        bases = [cx.eng.plan(dev, cfg) for _ in range(ns)]
        att = [b.attach(ScanConfig(n1p=POP, n2p=POP, window=500_000, fst=True, scan_wgs_per_cu=1)) for b in bases]
        rm = run_loop(cx, bases, args.steps, args.warmup, "config 3, 20 kb + 500 kb")
        w20 = n_windows(rm["gathered"])
        a0 = att[(args.steps - 1) % ns].read()
        w500 = int(((a0["flags"] & 0x80000000) == 0).sum())
        ms = rm["dt"] / args.steps * 1e3
        bpm = algorithmic_bytes(p.n, 0, w20 + w500, "pipeline")
        extra["config3_20kb_500kb"] = {
            "ms_per_step": ms, "windows_20kb": w20, "windows_500kb": w500,
            "windows_per_s": (w20 + w500) / (ms * 1e-3),
            "roofline_pipeline": {"achieved": bpm / (ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                  "frac": bpm / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "note": "BASELINE configs[2]'s two window sizes per step: one k_prep pass, the 500 kb plan attached to "
                    "the 20 kb base (its slots by binary search on the resident positions), both scans with "
                    "Fst; 2 plans on 2 streams as the headline loop"}
        for b in bases:
            b.close()
    nrec, grids, kname = plans[0].nrec, plans[0].grids(), plans[0].scan_kernel()
    for x in plans:
        x.close()
    dev.close()
    step_s = r["dt"] / args.steps
    out = {"value": total_windows * args.steps / r["dt"], "ms_per_step": step_s * 1e3,
           "gathered_info": ({"tables_gathered": r["gathers"] * r["group"], "passes_per_gather": r["group"],
                              "bytes_per_pass_all_ranks": r["gathered_bytes_per_pass"],
                              "windows_per_pass": total_windows} if cx.world > 1 else None),
           "host_enqueue_ms_per_step": r["t_enq"] / args.steps * 1e3,
           "device_ms_per_step": r["device_ms"] / args.steps, "gather_ms": r["gather_ms"],
           "settle": {"seconds": SETTLE_S, "passes": r["settle_passes"],
                      "note": "untimed passes before the warmup so that the timed steps run at the sustained clock"},
           "windows": total_windows, "snps": p.n, "cuts": cuts,
           "rank0": {"snps": sub.n, "windows": win_rank, "slots": nrec,
                     "k_prep_ms": r["k_timed_ms"][0], "scan_ms": r["k_timed_ms"][1],
                     "timed_samples": r["k_timed_samples"], "k_prep_alone_ms": k1, "scan_alone_ms": k3,
                     "dense_samples": dense and dense[2], "k_prep_dense_ms": dense and dense[0],
                     "scan_dense_ms": dense and dense[1],
                     "scan_kernel": kname, "single_stream_pass_ms": one,
                     "single_stream_pass_windows_per_s": win_rank / (one * 1e-3) if one else None,
                     "scan_grid_threads": grids[1]}}
    out.update(extra)
    return out, p


def config2_weak(cx, args):
    """BASELINE configs[1]: one 1e6-SNP chromosome per rank (seed 12345 + rank), 3 plans on 3 streams."""
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(1, C2_SNP, POP, POP, seed=C2_SEED + cx.rank)
    dev = cx.eng.upload(p)
    cfg = ScanConfig(n1p=POP, n2p=POP, window=WS, fst=True)
    ns = max(1, args.streams)
    steps = max(args.steps, args.config2_steps)
    gr = 0
    if cx.world > 1:   # every pass's table gathered, groups of P passes over the ns streams
        P = next(k for k in (args.group, 4, 2, 1) if k >= 1 and steps % k == 0)
        plans = [cx.eng.plan(dev, cfg) for _ in range(max(P, ns))]
        r = run_loop_gathered(cx, plans, steps, max(args.warmup, 20), "config 2", nstreams=ns)
    else:
        plans = [cx.eng.plan(dev, cfg) for _ in range(ns)]
        gr = 2 * ns * args.config2_graph if args.config2_graph > 0 else 0
        if gr:
            steps = -(-steps // gr) * gr
        r = run_loop(cx, plans, steps, max(args.warmup, 20), "config 2", graph_runs=gr)
    k1, k2, k3 = kernel_times(plans[0])
    one = single_pass_ms(cx, plans[0], 40) if cx.rank == 0 else None
    nrec, grids, kname = plans[0].nrec, plans[0].grids(), plans[0].scan_kernel()
    for x in plans[::-1]:
        x.close()
    dev.close()
    total = r.get("windows_per_pass_gathered") or n_windows(r["gathered"])
    nwin = n_windows(r["mine"])
    b3 = algorithmic_bytes(p.n, nrec, nwin, "k3")
    ach = b3 / (k3 * 1e-3) / 1e9
    traffic, tsrc = pmc_traffic(kname, grids[1])
    return {"value": total * steps / r["dt"], "unit": "windows/s", "scaling": "weak", "steps": steps,
            "ms_per_step": r["dt"] / steps * 1e3, "host_enqueue_ms_per_step": r["t_enq"] / steps * 1e3,
            "single_stream_pass_ms": one,
            "workload": "configs[1]: synthetic 1 chromosome x 1e6 SNPs per GPU (seed 12345 + rank), 20 kb, "
                        "per-chromosome background, T2D + T1D + Fst",
            "windows_per_gpu": nwin, "windows_all_gpus": total,
            "parallelism": f"one chromosome per GPU, {len(plans)} plans on {ns} HIP streams (passes overlap)"
                           + (f"; replayed as a HIP graph of {gr} runs" if cx.world == 1 and gr else "")
                           + ("; every pass's table (records + Fst) all-gathered over RCCL, overlapped with the "
                              f"next passes (groups of {r.get('group')})" if cx.world > 1 else ""),
            "kernels_ms": {"k_prep": k1, "k_bg_slice": k2, kname: k3},
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                         "traffic": traffic, "kernel": kname, "ms": k3, "algorithmic_bytes": b3,
                         "note": "the 8 MB stream is MALL-resident: not an HBM measurement; traffic: "
                                 + (tsrc or "no PMC pass committed")}}


C4_REP, C4_GEN, C4_WIN, C4_POP, C4_SEED = 2500, 4, 2000, 50, 20251016


def config4_sims(cx, args):
    """BASELINE configs[3]: sims_scan.likelihood_scan (sims_scan.py:593-644 -> process_window 451-590) over
    4 generations x 2,500 replicates x 2,000 windows of 20 kb (Poisson(358.5) SNPs per window: 7.17e9
    SNPs, 57 GB packed, generated in HBM by k_synth_sims), pop_size 50/50 (101 x 101 grid: k_scan_gw),
    each generation scanned against its own background (all its SNPs with pos in [0, 500000]: 2D
    folded, 1D unfolded -- quirk Q7).  The slot table comes from k_prep's segmentation of the resident
    positions, as real replicate VCFs need (not the generator's window offsets).  A step = one pass over
    all four generations: the four independent plans go round-robin on 2 HIP streams, so one
    generation's segmentation (bandwidth-bound) runs beside another's scan (latency-bound).  Inputs
    resident in HBM; generation time reported apart."""
    from sfs2d import _lib as L
    from sfs2d.engine import Plan, ScanConfig
    from sfs2d.synth import miss_table, sims_window_counts
    torch = cx.torch
    n, ws = C4_POP, WS
    mt = miss_table(2 * n)
    datas, plans, nsnp, t_gen = [], [], 0, 0.0
    prev = os.environ.get("SFS2D_SEG")
    # the slot table real replicate VCFs get: a binary search on the resident positions (k_slots_search),
    # not the generator's window offsets
    os.environ["SFS2D_SEG"] = args.c4_seg
    try:
        for g in range(C4_GEN):
            wc = sims_window_counts(C4_SEED, g, C4_REP, C4_WIN)
            nsnp += int(wc.astype(np.int64).sum())
            t0 = time.perf_counter()
            dev = cx.eng.synth_sims(C4_SEED, g, C4_REP, C4_WIN, ws, n, n, wc, mt, mt)
            torch.cuda.synchronize()
            t_gen += time.perf_counter() - t0
            h2, u1, u2 = cx.eng.bg_hist(dev, ScanConfig(n1p=n, n2p=n, start_position=0, end_position=500000), -1)
            pl = cx.eng.plan(dev, ScanConfig(n1p=n, n2p=n, window=ws, bg_mode=L.BG_SUPPLIED))
            pl.set_background(h2.reshape(-1).astype(np.float64), u1[: n + 1].astype(np.float64),
                              u2[: n + 1].astype(np.float64))
            datas.append(dev)
            plans.append(pl)
    finally:
        if prev is None:
            os.environ.pop("SFS2D_SEG", None)
        else:
            os.environ["SFS2D_SEG"] = prev
    kname, grids = plans[0].scan_kernel(), plans[0].grids()
    streams = [cx.streams[j % 2] for j in range(C4_GEN)]
    # one generation alone on one stream (a user scanning one generation's replicates)
    one = single_pass_ms(cx, plans[0], runs=5)
    k1a, _, k3a = kernel_times(plans[0], runs=4)
    for q in plans:
        q.run()
    torch.cuda.synchronize()
    t_s = time.perf_counter()
    while time.perf_counter() - t_s < SETTLE_S:
        Plan.run_streams(plans, streams, C4_GEN, None)
        torch.cuda.synchronize()
    steps = max(2, min(args.steps, args.sims_steps))
    for q in plans:
        q.set_timing(steps, every=1, kernels=5)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    Plan.run_streams(plans, streams, C4_GEN * steps, None)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kt = [q.timing_read() for q in plans]
    for q in plans:
        q.set_timing(0)
    nk = sum(c for c, _ in kt)
    k1 = sum(c * k[0] for c, k in kt) / max(1, nk)
    k3 = sum(c * k[2] for c, k in kt) / max(1, nk)
    nwin, nslot = 0, 0
    for q in plans:
        q.check()
        recs = q.read()
        nwin += int(((recs["flags"] & L.W_EMPTY) == 0).sum())
        nslot += q.nrec
    ms = dt / steps * 1e3
    b3 = algorithmic_bytes(nsnp // C4_GEN, nslot // C4_GEN, 0, "k3") - 24 * (nslot // C4_GEN)   # no Fst
    b3a = b3
    for q in plans:
        q.close()
    for d in datas:
        d.close()
    torch.cuda.synchronize()
    return {"value": nwin / (ms * 1e-3), "unit": "windows/s", "ms_per_step": ms, "steps": steps,
            "windows": nwin, "snps": nsnp, "generations": C4_GEN, "replicates": C4_REP,
            "workload": f"configs[3]: sims_scan likelihood_scan, {C4_GEN} generations x {C4_REP} replicates x "
                        f"{C4_WIN} windows of 20 kb, Poisson(358.5) SNPs per window ({nsnp} SNPs, "
                        f"{nsnp * 8 / 1e9:.1f} GB resident), pop_size 50/50 (101 x 101 grid), supplied per-generation "
                        "background; the slot table from the resident positions (no generator knowledge)",
            "parallelism": f"{C4_GEN} plans (one per generation) round-robin on 2 HIP streams",
            "generate_s": t_gen,
            "one_generation_alone_ms": one, "one_generation_alone_windows_per_s": (nwin / C4_GEN) / (one * 1e-3),
            "slot_table": {"search": "k_slots_search (binary search on the positions)",
                           "prep": "k_prep's segmentation pass"}.get(args.c4_seg, args.c4_seg),
            "kernels_ms": {"slots": k1, kname: k3, "alone": {"slots": k1a, kname: k3a}},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": b3 / (k3 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": b3 / (k3 * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": b3,
                         "frac_alone": b3a / (k3a * 1e-3) / 1e9 / HBM_PEAK_GBS, "scan_grid_threads": grids[1],
                         "note": "4 B/SNP + 72 B/slot (8-B slot record in, 64-B record out) per generation over the "
                                 "kernel's average duration in the timed steps (events in its dispatch packets, "
                                 "overlapped with the other stream's k_prep); frac_alone: one stream"}}


def config5_snpwin(cx, args):
    """BASELINE configs[4]: scan_perChr_bySNPs (twoDSFS_class.py:1422-1541) -- 500-SNP windows, pop_size
    100/75 (201 x 151 grid: k_scan_gw), per-chromosome backgrounds, T2D + T1D in fp64 (the tolerance
    sweep showed fp32 misses 1e-10: DESIGN.md), on 1e6 synthetic SNPs (4 chromosomes).  Passes overlapped
    on 2 HIP streams as the headline loop."""
    from sfs2d.engine import ScanConfig
    from sfs2d import _lib as L
    from sfs2d.synth import synth_genome
    p = synth_genome(4, 250_000, 100, 75, seed=2024)
    dev = cx.eng.upload(p)
    cfg = ScanConfig(n1p=100, n2p=75, window_mode=L.WINDOW_SNPS, window=500)
    plans = [cx.eng.plan(dev, cfg) for _ in range(2)]
    steps = max(args.steps, 200)
    r = run_loop(cx, plans, steps, max(args.warmup, 20), "config 5", time_kernels=True)
    k1, _, k3 = kernel_times(plans[0])
    one = single_pass_ms(cx, plans[0], 40)
    nrec, grids, kname = plans[0].nrec, plans[0].grids(), plans[0].scan_kernel()
    for q in plans:
        q.close()
    dev.close()
    nwin = n_windows(r["mine"])
    ms = r["dt"] / steps * 1e3
    b3 = 4 * p.n + (8 + 64) * nrec
    kt = r["k_timed_ms"][1]
    return {"value": nwin / (ms * 1e-3), "unit": "windows/s", "ms_per_step": ms, "steps": steps, "windows": nwin,
            "snps": p.n, "single_stream_pass_ms": one,
            "workload": "configs[4]: scan_perChr_bySNPs, 500-SNP windows, n1=200 n2=150 haploid (pop_size 100/75), "
                        "synthetic 4 chromosomes x 250,000 SNPs, per-chromosome backgrounds, T2D + T1D (fp64)",
            "parallelism": "2 plans on 2 HIP streams (passes overlap)",
            "kernels_ms": {"k_prep": k1, kname: k3, "timed_loop": {"k_prep": r["k_timed_ms"][0], kname: kt}},
            "roofline": {"bound": "hbm", "kernel": kname, "achieved": b3 / (kt * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": b3 / (kt * 1e-3) / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes": b3,
                         "scan_grid_threads": grids[1],
                         "note": "4 B/SNP + 72 B/slot over the kernel's average duration in the timed steps; the 4 MB "
                                 "stream is MALL-resident, so this is not an HBM measurement"}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the VCF -> CSV end-to-end timing")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 (weak scaling) key")
    ap.add_argument("--no-variants", action="store_true", help="skip the config-3 run without Fst")
    ap.add_argument("--streams", type=int, default=0,
                    help="config 2: plans / HIP streams (passes overlap); 0: 4 at N = 1 (replayed as HIP graphs), 3 at N > 1")
    ap.add_argument("--config2-steps", type=int, default=400, help="config 2: at least this many passes")
    ap.add_argument("--config2-graph", type=int, default=8,
                    help="config 2 at N = 1: k > 0 replays per-stream HIP graphs of 2 k runs per plan (Plan.graph), "
                         "0: run_streams")
    ap.add_argument("--no-sims", action="store_true", help="skip the config-4 / config-5 keys")
    ap.add_argument("--sims-steps", type=int, default=5, help="config 4: timed passes over the 4 generations")
    ap.add_argument("--c4-seg", default="search", choices=["search", "prep"],
                    help="config 4's slot table: binary search on the positions, or k_prep's segmentation")
    ap.add_argument("--group", type=int, default=4,
                    help="N > 1: passes per all-gather group (every pass's table is gathered; P must divide steps)")
    args = ap.parse_args()
    if args.gpus < 1 or args.steps < 1:
        raise SystemExit("--gpus and --steps must be >= 1")
    # hardware queues per process: HIP maps streams onto GPU_MAX_HW_QUEUES queues (4 on the box); the
    # pass streams + the library's and torch's own need more than 4 or two passes share a queue and
    # serialise (profiles/r02h_*).  Set before the HIP runtime starts (rank processes inherit it).
    if args.streams <= 0:
        # config 2, measured at N = 1 (profiles/r06ad3*): 4 streams replayed as graphs 2.65-2.75e8
        # windows/s, 3 streams 2.41e8, 2 1.97e8, 5-6 1.4-1.6e8; without graphs 4 streams are host-bound
        # (2.30-2.63e8).  N > 1 keeps the 3 measured with the all-gather stream beside them.
        args.streams = 4 if args.gpus == 1 else 3
    need = max(2, args.streams) + 4
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
    if SHARED_GPU:
        local = 0   # rehearsal of the N > 1 code path on a one-GPU box: not a scaling measurement
    elif ndev < world or local >= ndev:
        raise RuntimeError(f"bench.py --gpus {world}: rank {rank} needs device {local}, {ndev} visible")
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        dist.init_process_group("gloo" if SHARED_GPU else "nccl", rank=rank, world_size=world)
        world = dist.get_world_size()   # n_gpus from the communicator
    cx = Ctx(world, rank, local, max(2, args.streams))

    c3, genome = config3_strong(cx, args)
    c2 = None if args.no_config2 else config2_weak(cx, args)
    c4 = c5 = None
    if world == 1 and not args.no_sims:
        c5 = config5_snpwin(cx, args)
        c4 = config4_sims(cx, args)

    if rank == 0:
        r0 = c3["rank0"]
        b3 = algorithmic_bytes(r0["snps"], r0["slots"], r0["windows"], "k3")
        ach = b3 / (r0["scan_ms"] * 1e-3) / 1e9
        bp = algorithmic_bytes(c3["snps"], 0, c3["windows"], "pipeline")
        step_s = c3["ms_per_step"] * 1e-3
        traffic, tsrc = pmc_traffic(r0["scan_kernel"], r0["scan_grid_threads"])
        line = {
            "metric": METRIC, "value": c3["value"], "unit": "windows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": c3["ms_per_step"], "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (SURVEY 8d generator, seed 777)",
            "config": {"workload": "configs[2]: synthetic whole genome, 32 chromosomes x 1.5625e6 = 5e7 SNPs, 20 kb "
                                   "windows, n1=n2=50 haploid (pop_size 25/25), per-chromosome background, "
                                   "sharded by window over the GPUs",
                       "snps": c3["snps"], "windows": c3["windows"], "window_bp": WS,
                       "stats": "T2D, T1D_p1, T1D_p2 (reference semantics) + Hudson Fst (DESIGN.md; not in the "
                                "reference, parity vs its own oracle restatement)",
                       "parallelism": f"{world} GPU(s), SNP ranges cut at window starts ({c3['cuts']}: chromosome "
                                      "ends, no background exchange); passes overlapped on 2 HIP streams per GPU"
                                      + ("; EVERY pass's window table (64-B records + 8-B Fst) all-gathered to every "
                                         "rank over RCCL inside the timed region, each group's gather overlapped with "
                                         "the next group's passes; value counts gathered windows only"
                                         if world > 1 else "")},
            "host_enqueue_ms_per_step": c3["host_enqueue_ms_per_step"],
            "device_ms_per_step": c3["device_ms_per_step"], "gather_ms": c3["gather_ms"],
            "gather_ms_per_step": (c3["gather_ms"] / args.steps) if world > 1 else None,
            "gathered": c3.get("gathered_info"), "settle": c3["settle"],
            "rank0": r0,
            "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "kernel": r0["scan_kernel"],
                         "ms": r0["scan_ms"], "algorithmic_bytes": b3,
                         "note": r0["scan_kernel"] + " on rank 0's shard: 4 B/SNP + 96 B/slot per launch over its average "
                                 "duration in the timed steps (start / end events in the kernels' dispatch packets, "
                                 "2 timed passes per plan, overlapped with the other stream's k_prep; alone on one "
                                 "stream: rank0.scan_alone_ms); traffic: " + (tsrc or "no PMC pass committed"),
                         "dense_check": ({"ms": r0["scan_dense_ms"], "launches": r0["dense_samples"],
                                          "frac": b3 / (r0["scan_dense_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                          "note": "the same kernel over 10 more untimed loops of the timed loop's "
                                                  "passes, plans, streams and sampling (dense_kernel_samples)"}
                                         if r0.get("scan_dense_ms") else None)},
            "roofline_pipeline": {"bound": "hbm", "achieved": bp / step_s / 1e9, "peak": HBM_PEAK_GBS * world,
                                  "unit": "GB/s", "frac": bp / step_s / 1e9 / (HBM_PEAK_GBS * world),
                                  "note": "whole step over all GPUs (SURVEY 8(d): 12 B/SNP + 64 B/window) over "
                                          "ms_per_step"},
        }
        if "t2d_t1d_only" in c3:
            line["t2d_t1d_only"] = c3["t2d_t1d_only"]
            line["fst_cost"] = c3["fst_cost_interleaved"]
        if "config3_20kb_500kb" in c3:
            line["config3_20kb_500kb"] = c3["config3_20kb_500kb"]
        if c2 is not None:
            line["config2_weak"] = c2
        if c4 is not None:
            line["config4_sims"] = c4
        if c5 is not None:
            line["config5_snp_windows"] = c5
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(genome.subset_chroms([0]))
        if not args.no_e2e and world == 1:
            line["end_to_end_vcf_csv"] = end_to_end()
        if SHARED_GPU and world > 1:
            line["shared_gpu_rehearsal"] = "SFS2D_BENCH_SHARED_GPU: every rank on GPU 0 over gloo -- a code-path check, not a measurement"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
