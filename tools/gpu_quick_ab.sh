#!/bin/bash
# quick check of a kernel change: GPU parity subset, then per-kernel timings of config 2 / config 3
# (with and without Fst).  usage: bash tools/gpu_quick_ab.sh <tag> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
K=${2:-"parity or fst or multires or config"}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "$K" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for C in "config3 30 fst" "config3 30" "config2 30 fst"; do
    echo -n "$C: " >> $OUT/ab.log
    timeout -k 10 120 python tools/profile_scan.py $C 2>&1 | grep nrec >> $OUT/ab.log || exit 1
  done
done
cat $OUT/ab.log
