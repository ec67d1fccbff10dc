#!/bin/bash
# round 3: Fst (p, A) table in k_prep -- GPU tests, A/B timing, bench
set -o pipefail
OUT=gpurun_out/r03e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 450 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
for r in 1 2; do
  for t in 0 1; do
    for c in config2 config3; do
      echo -n "notab=$t " >> $OUT/ab.log
      if [ $t = 1 ]; then export SFS2D_NO_FST_TAB=1; else unset SFS2D_NO_FST_TAB; fi
      timeout -k 10 120 python tools/profile_scan.py $c 30 fst 2>&1 | grep nrec >> $OUT/ab.log || exit 1
    done
  done
done
unset SFS2D_NO_FST_TAB
cat $OUT/ab.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-1500
