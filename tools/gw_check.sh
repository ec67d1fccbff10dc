#!/bin/bash
# Large-grid kernels: parity tests, then k_scan_gw vs k_scan_g on config 4 (one generation) and config 5.
# usage: bash tools/gw_check.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-gw}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:-"large_grid or sims or fst_vs_oracle or records_per_chrom or synth"}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for gw in 1 0; do
  SFS2D_GW=$gw timeout -k 10 240 python -u tools/sims_config4.py 2500 1 5 >> $OUT/config4.log 2>&1 || { cat $OUT/config4.log; exit 1; }
  SFS2D_GW=$gw timeout -k 10 180 python -u tools/profile_scan.py config5 20 fst >> $OUT/config5.log 2>&1 || { cat $OUT/config5.log; exit 1; }
done
cat $OUT/config4.log $OUT/config5.log
