#!/bin/bash
# Quick GPU check: parity tests + per-config kernel timings (Fst on).  usage: bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
TAG=${1:-q}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:-}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for c in config2 config3 config5; do
  timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> $OUT/profile_scan.log 2>&1 || { cat $OUT/profile_scan.log; exit 1; }
done
cat $OUT/profile_scan.log
