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


@pytest.mark.timeout(300)
def test_single_chromosome_split_two_ranks_equals_one_rank(tmp_path):
    """One chromosome split over 2 ranks (HIP plans, k_prep -> background all-reduce -> scan):
    the merged table equals one rank's whole-chromosome table byte for byte."""
    got = run_dist_workers("gpu", 2, str(tmp_path / "out.json"), extra=("single",), timeout=240)
    check_single(got)
