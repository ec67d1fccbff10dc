#!/usr/bin/env python3
"""Benchmark: genomic windows/s of the 2D-SFS composite-likelihood scan (BASELINE.json metric).

Workload (BASELINE configs[1]): one synthetic chromosome of 1e6 SNPs per GPU (SURVEY 8d
generator, seed 12345 + rank), n1 = n2 = 50 haploid (pop_size 25/25), 20 kb fixed-bp windows,
each chromosome its own background (combined_scan semantics).  A step = one full scan pass over
the HBM-resident packed SNPs: background histograms + window segmentation (K1), background
tables (K2), window scan (K3) -> device-resident 64-B window records; with N > 1 ranks, plus one
RCCL all-gather of every rank's window table (weak scaling: per-GPU work fixed).

Prints ONE JSON line on rank 0.  `roofline` is for the dominant kernel (K3) from HIP events on
the stream the kernels run on, during the timed steps; `roofline_hbm` repeats the measurement
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
    """Bytes each kernel must move (DESIGN.md "Kernels"): k_prep reads counts + positions (8 B/SNP),
    writes the packed bins (4 B/SNP) and the window slot table (8 B/window); k_scan_w reads the bins
    (4 B/SNP) and the slot table (8 B/slot) and writes one 64-B record per slot."""
    if which == "k3":
        return 4 * n_snp + 8 * n_slots + 64 * n_slots
    if which == "k1":
        return 12 * n_snp + 8 * n_win
    return 16 * n_snp + 8 * n_win + 72 * n_slots


def cpu_baseline(p):
    """Oracle (numpy/scipy restatement of the reference's dense per-window algorithm, test
    infrastructure only) over the whole rank-0 config-2 stream, one host core."""
    from oracle import sfs_oracle as O
    cfg = O.Cfg(POP, POP)
    t0 = time.perf_counter()
    res = O.combined_scan(p, WS, cfg)
    dt = time.perf_counter() - t0
    return {"value": len(res) / dt, "unit": "windows/s", "cores": 1, "kind": "port",
            "sample": f"the full rank-0 config-2 stream ({p.n} SNPs, {len(res)} windows, {dt:.1f} s): "
                      "oracle/sfs_oracle.combined_scan, dense per-window grids + scipy multinomial.logpmf "
                      "as the reference computes them, single thread"}


def hbm_stream_roofline(eng, steps=5):
    """BASELINE config 3 on one GPU (5e7 SNPs, 32 chromosomes, ~600 MB read): past the MALL."""
    from sfs2d.engine import ScanConfig
    from sfs2d.synth import synth_genome
    p = synth_genome(32, 1_562_500, POP, POP, seed=777)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=POP, n2p=POP, window=WS))
    pl.run()
    pl.check()
    pl.set_timing(steps, every=2)
    pl.run_many(2 * steps)
    nr, (k1, k2, k3) = pl.timing_read()
    recs = pl.read()
    nwin = int(((recs["flags"] & 0x80000000) == 0).sum())
    b3 = algorithmic_bytes(p.n, pl.nrec, nwin, "k3")
    b1 = algorithmic_bytes(p.n, pl.nrec, nwin, "k1")
    out = {"bound": "hbm", "achieved": b3 / (k3 * 1e-3) / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": b3 / (k3 * 1e-3) / 1e9 / HBM_PEAK_GBS, "kernel": "k_scan", "ms": k3,
           "k1_GBs": b1 / (k1 * 1e-3) / 1e9, "k1_ms": k1, "k2_ms": k2,
           "pipeline_GBs": algorithmic_bytes(p.n, pl.nrec, nwin, "all") / ((k1 + k2 + k3) * 1e-3) / 1e9,
           "windows": nwin, "windows_per_s": nwin / ((k1 + k2 + k3) * 1e-3),
           "workload": "config 3 stream on 1 GPU: 32 chrom x 1.5625e6 SNPs, 20 kb, per-chromosome bg"}
    pl.close()
    dev.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hbm-stream", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world)
    torch.cuda.set_device(local)

    from sfs2d import _lib as L
    from sfs2d.engine import Engine, ScanConfig
    from sfs2d.synth import synth_genome

    p = synth_genome(1, N_SNP, POP, POP, seed=12345 + rank)
    eng = Engine.get(local)
    stream = torch.cuda.Stream(device=local)   # one stream shared by the HIP library and torch/RCCL
    torch.cuda.set_stream(stream)
    eng.set_stream(stream.cuda_stream)
    dev = eng.upload(p)
    pl = eng.plan(dev, ScanConfig(n1p=POP, n2p=POP, window=WS))
    nrec = pl.nrec
    out = torch.empty((nrec, 64), dtype=torch.uint8, device=f"cuda:{local}")
    gathered = None
    if world > 1:
        gathered = torch.empty((world, nrec, 64), dtype=torch.uint8, device=f"cuda:{local}")
        counts = torch.tensor([nrec], device=f"cuda:{local}")
        allc = [torch.zeros_like(counts) for _ in range(world)]
        dist.all_gather(allc, counts)
        assert all(int(c) == nrec for c in allc), "weak-scaling shards must have equal record counts"

    def step():
        pl.run(out.data_ptr())
        if world > 1:
            dist.all_gather_into_tensor(gathered.view(world * nrec, 64), out)

    pl.run(out.data_ptr())
    pl.check()
    for _ in range(args.warmup):
        step()
    # HIP events around each kernel of every 8th timed run, on the stream the kernels run on (sampled:
    # an event pair costs several microseconds of queue time, 1/8 of it is ~1 us per step)
    pl.set_timing(args.steps, every=8)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if world == 1:
        pl.run_many(args.steps, out.data_ptr())   # enqueued from C: no host work between steps
    else:
        for _ in range(args.steps):
            step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    nr, (k1, k2, k3) = pl.timing_read()
    pl.check()
    recs = np.frombuffer(out.cpu().numpy().tobytes(), dtype=L.WINDOW_DTYPE)
    nwin_rank = int(((recs["flags"] & L.W_EMPTY) == 0).sum())
    total_windows = nwin_rank * world
    value = total_windows * args.steps / dt

    if rank == 0:
        b3 = algorithmic_bytes(p.n, nrec, nwin_rank, "k3")
        achieved = b3 / (k3 * 1e-3) / 1e9
        line = {
            "metric": "genomic windows/s (T2D+T1D_p1+T1D_p2; Fst not computed yet) at 20 kb, n1=n2=50",
            "value": value, "unit": "windows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic (SURVEY 8d generator, seed 12345+rank)",
            "config": {"workload": "configs[1]: synthetic 1 chromosome x 1e6 SNPs per GPU, 20 kb windows, "
                                   "n1=n2=50 haploid (pop_size 25/25), per-chromosome background",
                       "snps_per_gpu": p.n, "windows_per_gpu": nwin_rank, "window_bp": WS,
                       "parallelism": f"windows sharded by chromosome over {world} GPU(s); RCCL all-gather"},
            "kernels_ms": {"k_prep": k1, "k_bg_slice_or_gap": k2, "k_scan_w": k3, "timed_runs": nr,
                           "exact_path_windows": pl.stats()},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "k_scan_w", "ms": k3,
                         "note": "k_scan_w, algorithmic bytes 4 B/SNP + 72 B/slot per launch over its event-timed "
                                 "duration; the 8 MB config-2 stream is MALL-resident (see roofline_hbm)"},
        }
        if not args.no_hbm_stream and world == 1:
            line["roofline_hbm"] = hbm_stream_roofline(eng)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(p)
        print(json.dumps(line), flush=True)
    pl.close()
    dev.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
