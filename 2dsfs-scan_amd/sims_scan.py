"""Drop-in replacement for the reference module ``scripts/sims_scan.py`` (simulation scans).

Functional API of sims_scan.py:18-690 for the window-scan path.  Differences from the class
API that the reference has and that are kept:
* no None guards: an empty window or background raises ZeroDivisionError (325-440);
* the 1D backgrounds passed to ``process_window`` are read at raw keys 1..pop_size-1 (the
  sims driver hands it UNFOLDED spectra, 615-617);
* ``T2D_diff = T2D - (T1D_p1 - T1D_p2)/2`` (minus; 497, 538, 573);
* records carry window_type / window_start / window_end.
All statistics come from the HIP kernels (sfs2d.engine); no CPU fallback.
"""
from __future__ import annotations

import csv
import glob
import os

import numpy as np

from sfs2d import _lib as L
from sfs2d import post
from sfs2d.engine import Engine, ScanConfig
from sfs2d.vcf import make_data_dict_vcf  # noqa: F401  (sims_scan.py:18-120)
from sfs2d.pack import PackedSNPs, pack_snp_dict

_NO_ANN = 1 << 20
DEVICE = int(os.environ.get("SFS2D_DEVICE", "0"))


def _pack(data, pop1, pop2):
    return data if isinstance(data, PackedSNPs) else pack_snp_dict(data, pop1, pop2)


def _ann(p, variant_type):
    if variant_type is None:
        return -1
    return p.ann_names.index(variant_type) if variant_type in p.ann_names else _NO_ANN


def _hist(data, pop1, pop2, n1p, n2p, start_position, end_position, variant_type, fold):
    p = _pack(data, pop1, pop2)
    if pop1 == pop2:
        p = p.single_pop(pop1)
    n1, n2 = 2 * n1p, 2 * n2p
    if p.n == 0:
        return np.zeros((n1 + 1, n2 + 1), np.int64), np.zeros(n1 + 1, np.int64), np.zeros(n2 + 1, np.int64)
    eng = Engine.get(DEVICE)
    dev = eng.upload(p)
    cfg = ScanConfig(n1p=n1p, n2p=n2p, fold=fold, ann_want=_ann(p, variant_type),
                     start_position=None if start_position is None else int(start_position),
                     end_position=None if end_position is None else int(end_position))
    try:
        return eng.bg_hist(dev, cfg, -1)
    finally:
        dev.close()


def calculate_2d_sfs(data_dict, pop1, pop2, pop1_size, pop2_size, start_position, end_position, variant_type,
                     fold=True):
    """sims_scan.py:123-234 (GPU histogram)."""
    h2, _, _ = _hist(data_dict, pop1, pop2, pop1_size, pop2_size, start_position, end_position, variant_type, fold)
    return {(i, j): int(h2[i, j]) for i in range(2 * pop1_size + 1) for j in range(2 * pop2_size + 1)}


def calculate_1d_sfs(data_dict, pop, pop_size, start_position, end_position, variant_type):
    """sims_scan.py:262-302 (GPU histogram, unfolded)."""
    _, u1, _ = _hist(data_dict, pop, pop, pop_size, pop_size, start_position, end_position, variant_type, False)
    return {i: int(u1[i]) for i in range(2 * pop_size + 1)}


def fold_1d_sfs(sfs_dict):
    """sims_scan.py:305-322."""
    num_chromosomes = max(sfs_dict.keys())
    folded = {}
    for freq, count in sfs_dict.items():
        m = min(freq, num_chromosomes - freq)
        folded[m] = folded[m] + count if m in folded else count
    return folded


def normalize_2d_sfs(sfs):
    """sims_scan.py:236-249."""
    counts = list(sfs.values())
    total = sum(counts[1:-1])
    return {k: v / total for k, v in sfs.items()}


def count_snps(window_data, variant_type):
    """sims_scan.py:251-259."""
    if variant_type is None:
        return len(window_data)
    return sum(1 for d in window_data.values() if d.get("annotation") == variant_type)


def calculate_likelihood_1D(foreground_sfs, background_sfs):
    """sims_scan.py:325-395 (no guards)."""
    from sfs2d.dense import clr_1d
    return clr_1d(Engine.get(DEVICE), foreground_sfs, background_sfs, guards=False)


def calculate_likelihood_2D(foreground_2d_sfs, background_2d_sfs):
    """sims_scan.py:398-440 (no guards)."""
    from sfs2d.dense import clr_2d
    return clr_2d(Engine.get(DEVICE), foreground_2d_sfs, background_2d_sfs, guards=False)


def get_gens(main_dir):
    """sims_scan.py:442-449: generation ids = 2nd dot-field of 5-field file names."""
    search_strings = set()
    for root, dirs, files in os.walk(main_dir):
        for file in files:
            parts = file.split('.')
            if len(parts) == 5:
                search_strings.add(parts[1])
    return search_strings


def _bg_arrays(bg_2d_sfs, bg_p1_sfs, bg_p2_sfs, pop1_size, pop2_size):
    n1, n2 = 2 * pop1_size, 2 * pop2_size
    keys = [(i, j) for i in range(n1 + 1) for j in range(n2 + 1)]
    b2 = np.zeros(len(keys), np.float64)
    for k, key in enumerate(keys[1:-1], start=1):
        b2[k] = bg_2d_sfs[key]
    b1 = np.zeros(pop1_size + 1, np.float64)
    b1b = np.zeros(pop2_size + 1, np.float64)
    for k in range(1, pop1_size):
        b1[k] = bg_p1_sfs[k]
    for k in range(1, pop2_size):
        b1b[k] = bg_p2_sfs[k]
    return b2, b1, b1b


def process_window(data_dict, bg_2d_sfs, bg_p1_sfs, bg_p2_sfs, window_size, pop1, pop2, pop1_size, pop2_size,
                   start_position, end_position, variant_type):
    """sims_scan.py:451-590: fixed-bp windows against one supplied background."""
    p = _pack(data_dict, pop1, pop2)
    eng = Engine.get(DEVICE)
    cfg = ScanConfig(n1p=pop1_size, n2p=pop2_size, fold=True, window_mode=L.WINDOW_BP, window=window_size,
                     bg_mode=L.BG_SUPPLIED, ann_want=_ann(p, variant_type),
                     start_position=None if start_position is None else int(start_position),
                     end_position=None if end_position is None else int(end_position))
    bg = _bg_arrays(bg_2d_sfs, bg_p1_sfs, bg_p2_sfs, pop1_size, pop2_size)
    dev = eng.upload(p)
    try:
        recs = eng.scan(dev, cfg, bg)
    finally:
        dev.close()
    return post.sims_process_window(recs, p, window_size, post.num_slots(recs))


def _concat(packs):
    """Replicates -> one packed data set (each replicate's chromosomes one after the other; the
    annotation tables merged).  Returns the data set and each replicate's first chromosome index."""
    names, counts, pos, ann, offs, base = [], [], [], [], [0], []
    ann_names, ann_ix = [], {}
    for q in packs:
        base.append(len(names))
        names.extend(q.chrom_names)
        counts.append(q.counts)
        pos.append(q.pos)
        remap = np.zeros(max(1, len(q.ann_names)), np.uint16)
        for i, a in enumerate(q.ann_names):
            if a not in ann_ix:
                ann_ix[a] = len(ann_names)
                ann_names.append(a)
            remap[i] = ann_ix[a]
        ann.append(remap[q.ann_id] if q.n else np.zeros(0, np.uint16))
        offs.extend((offs[-1] + q.chrom_off[1:]).tolist())
    cat = (lambda xs, dt: np.concatenate(xs) if xs else np.zeros(0, dt))
    return PackedSNPs(cat(counts, np.uint32), cat(pos, np.uint32), np.array(offs, np.int64), names,
                      cat(ann, np.uint16), ann_names), base


def _scan_local(p, cfg, bg):
    eng = Engine.get(DEVICE)
    dev = eng.upload(p)
    try:
        return eng.scan(dev, cfg, bg)
    finally:
        dev.close()


def _split_scan(p, cfg, bg):
    from sfs2d.engine import SplitJob
    return SplitJob(Engine.get(DEVICE), p, cfg, bg)


_split_scan.device_rows = True   # its jobs exchange background rows in HBM (sfs2d.dist._split_device)


def process_windows_batch(replicates, bg_2d_sfs, bg_p1_sfs, bg_p2_sfs, window_size, pop1, pop2, pop1_size,
                          pop2_size, start_position=None, end_position=None, variant_type=None, distributed=False):
    """``process_window`` (sims_scan.py:451-590) over many replicate data sets in ONE scan launch:
    all replicates resident in HBM as one data set, one supplied background, one plan.  Returns the
    list of per-replicate result dicts, each equal to ``process_window(replicate, ...)``; the first
    replicate (in order) whose window has no SNP / an empty background raises ZeroDivisionError, as
    the reference's loop over replicates would (sims_scan.py:619-622).  ``distributed``: the
    replicates' chromosomes are sharded over the torch.distributed group (one process per GPU, all
    ranks calling with the same arguments; every rank returns the whole list), split at window
    boundaries balanced by SNPs (sfs2d.dist.scan_records_split)."""
    packs = [_pack(d, pop1, pop2) for d in replicates]
    if not packs:
        return []
    data, base = _concat(packs)
    cfg = ScanConfig(n1p=pop1_size, n2p=pop2_size, fold=True, window_mode=L.WINDOW_BP, window=window_size,
                     bg_mode=L.BG_SUPPLIED, ann_want=_ann(data, variant_type),
                     start_position=None if start_position is None else int(start_position),
                     end_position=None if end_position is None else int(end_position))
    bg = _bg_arrays(bg_2d_sfs, bg_p1_sfs, bg_p2_sfs, pop1_size, pop2_size)
    if distributed:
        from sfs2d import dist as D
        recs = D.scan_records_split(data, cfg, bg, _split_scan, DEVICE)
    else:
        recs = _scan_local(data, cfg, bg)
    chrom = recs["chrom"].astype(np.int64)
    out = []
    for i, q in enumerate(packs):
        sel = (chrom >= base[i]) & (chrom < base[i] + q.nchrom)
        sub = recs[sel].copy()
        sub["chrom"] -= base[i]
        out.append(post.sims_process_window(sub, q, window_size, len(sub)))
    return out


def _generation_scans(main_dir, popinfo_filename, pop1, pop2, pop1_size, pop2_size, window_size, bg_end):
    """The loops shared by both ``likelihood_scan`` variants (sims_scan.py:607-622 / 657-671):
    yields (generation, iteration number, window coords, process_window result) in the reference's
    order -- generations in get_gens' set order, targets in glob order, windows in scan order.  Per
    generation, background = the concatenated VCF's SNPs with pos in [0, bg_end] (2D folded, 1D
    unfolded); the replicates of a generation are parsed by the native VCF reader and scanned in one
    launch (``process_windows_batch``)."""
    from sfs2d.vcf import read_vcf
    for generation in get_gens(main_dir):
        target_vcfs = glob.glob(f"{main_dir}/iter*/*{generation}*.vcf.gz")
        concatenated_vcfs = glob.glob(f"{main_dir}/concatenated_vcfs/gen.{generation}.concatenated.vcf.gz")
        for vcf in concatenated_vcfs:
            bgp = read_vcf(vcf, popinfo_filename).to_packed(pop1, pop2)
            bg_2d_sfs = calculate_2d_sfs(bgp, pop1, pop2, pop1_size, pop2_size, start_position=0,
                                         end_position=bg_end, variant_type=None)
            bg_p1_sfs = calculate_1d_sfs(bgp, pop1, pop1_size, start_position=0, end_position=bg_end,
                                         variant_type=None)
            bg_p2_sfs = calculate_1d_sfs(bgp, pop2, pop2_size, start_position=0, end_position=bg_end,
                                         variant_type=None)
            targets = [read_vcf(v, popinfo_filename).to_packed(pop1, pop2) for v in target_vcfs]
            batch = process_windows_batch(targets, bg_2d_sfs, bg_p1_sfs, bg_p2_sfs, window_size, pop1, pop2,
                                          pop1_size, pop2_size)
            for vcf_input, results in zip(target_vcfs, batch):
                iteration_number = int(vcf_input.split('.')[2])
                for window_coords, result in results.items():
                    yield generation, iteration_number, window_coords, result


def likelihood_scan(main_dir, output=None, popinfo_filename=None, pop1='p1', pop2='p2', pop1_size=5, pop2_size=5,
                    window_size=500000, bg_end=500000):
    """Both reference variants.  ``likelihood_scan(main_dir)`` (sims_scan.py:646-690, the definition
    the module keeps): returns {(generation, iteration, window_coords): {"generation", "iteration",
    "region", "window_coords", "likelihood": process_window's record}}.  With ``output``
    (sims_scan.py:593-644): writes the per-window CSV instead and returns None.  The reference
    hard-codes the popmap path and the sizes; here they are arguments (``popinfo_filename`` defaults
    to $SFS2D_SIMS_POPMAP; a missing file raises FileNotFoundError, as the reference's open of its
    absolute path does elsewhere)."""
    if popinfo_filename is None:
        popinfo_filename = os.environ.get("SFS2D_SIMS_POPMAP", "popmap_sims_copy.txt")
    if not os.path.exists(popinfo_filename):
        raise FileNotFoundError(f"[Errno 2] No such file or directory: '{popinfo_filename}'")
    scans = _generation_scans(main_dir, popinfo_filename, pop1, pop2, pop1_size, pop2_size, window_size, bg_end)
    if output is None:
        likelihood_results = {}
        for generation, iteration_number, key, value in scans:
            window_start, window_end = map(int, key.split(' ')[1].split('-'))
            region = 'background' if window_end <= 1000000 else 'foreground'
            likelihood_results[(generation, iteration_number, key)] = {
                'generation': generation, 'iteration': iteration_number, 'region': region,
                'window_coords': key, 'likelihood': value}
        return likelihood_results
    col_names = ['generation', 'iteration', 'region', 'window_coords', 'snp_count', 'T2D', 'T1D_p1', 'T1D_p2',
                 'new_term_p1', 'new_term_p2', 'T2D_diff']
    with open(output, 'w', newline='') as csvfile:
        writer = csv.DictWriter(csvfile, fieldnames=col_names)
        writer.writeheader()
        for generation, iteration_number, window_coords, result in scans:
            window_start, window_end = window_coords.split(' ')[1].split('-')
            region = 'background' if int(window_end) <= 1000000 else 'foreground'
            writer.writerow({'generation': generation, 'iteration': iteration_number, 'region': region,
                             'window_coords': window_coords, 'snp_count': result["snp_count"],
                             'T2D': result["T2D"], 'T1D_p1': result["T1D_p1"], 'T1D_p2': result["T1D_p2"],
                             'new_term_p1': result["new_term_p1"], 'new_term_p2': result["new_term_p2"],
                             'T2D_diff': result["T2D_diff"]})
    return None
