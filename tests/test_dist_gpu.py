"""The sharded HIP path at world > 1: two rank processes on the one GPU of the box (gloo group, each
rank its own HIP context), every golden driver call through the drop-in modules with
distributed=True, equal to the reference's outputs (tests/golden)."""
import pytest

from test_dist_cpu import check_dist_results, check_single, run_dist_workers

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(400)
def test_sharded_drivers_two_ranks_on_gpu(golden, tmp_path):
    got = run_dist_workers("gpu", 2, str(tmp_path / "out.json"), extra=("all",), timeout=360)
    assert check_dist_results(got, golden) >= 45
    # most calls (the sims batch included: its factory exchanges in HBM) ran split, not by the
    # whole-chromosome fallback (which only the error cases take)
    st = got["_stats"]
    assert st["split"] >= 30 and st["allreduce"] >= 10 and st["fallback"] <= 12, st


@pytest.mark.timeout(300)
def test_single_chromosome_split_two_ranks_equals_one_rank(tmp_path):
    """One chromosome split over 2 ranks (HIP plans, k_prep -> background all-reduce -> scan):
    the merged table equals one rank's whole-chromosome table byte for byte."""
    got = run_dist_workers("gpu", 2, str(tmp_path / "out.json"), extra=("single",), timeout=240)
    check_single(got)


@pytest.mark.timeout(900)
def test_config3_split_three_ranks_equals_one_gpu(tmp_path):
    """BASELINE config 3 at full size (5e7 SNPs) split over 3 rank processes on the box's GPU (cuts inside
    chromosomes: their background rows all-reduced from HBM): 20 kb and 500 kb per-chromosome scans and
    the genome-wide-background scan (sharded calculate_2d_sfs -> normalise -> scan_precomputed_BG) each
    equal, byte for byte, to one GPU's table over the whole genome."""
    import numpy as np
    from sfs2d.synth import synth_genome
    p = synth_genome(32, 1_562_500, 25, 25, seed=777)
    path = str(tmp_path / "cfg3.npz")
    np.savez(path, counts=p.counts, pos=p.pos, chrom_off=p.chrom_off)
    del p
    got = run_dist_workers("gpu", 3, str(tmp_path / "out.json"), extra=("config3", path), timeout=800)
    assert got["genome_hist_equal"], got
    cuts = got["cuts"]
    assert len(cuts) == 4 and 0 < cuts[1] < cuts[2] < 50_000_000
    for name in ("bp20k_perchrom", "bp500k_perchrom", "bp20k_genome_bg"):
        g = got[name]
        assert g["equal"] and g["split"] == 1, (name, g)
    assert got["bp20k_perchrom"]["windows"] > 130_000 and got["bp500k_perchrom"]["windows"] > 5_000


@pytest.mark.timeout(300)
def test_single_chromosome_split_rccl_world1(tmp_path):
    """The split path on an RCCL (nccl backend) group of one rank: the background rows all-reduced and
    the record tables all-gathered on device buffers by RCCL itself (the 2-rank tests above run gloo)."""
    got = run_dist_workers("gpu", 1, str(tmp_path / "out.json"), extra=("single",), timeout=240,
                           env_extra={"SFS2D_TEST_BACKEND": "nccl"})
    check_single(got)
