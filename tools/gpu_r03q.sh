#!/bin/bash
# k_prep loads one step ahead (default build) vs not (build/ab/lib_NOPF.so): parity subset, then timings
set -o pipefail
OUT=gpurun_out/r03q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "parity or fst or multires or config or sims or bg" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for r in 1 2; do
  for V in default NOPF; do
    for C in "config3 30" "config3 30 fst" "config2 30 fst"; do
      echo -n "$V $C: " >> $OUT/ab.log
      if [ $V = default ]; then unset SFS2D_LIB; else export SFS2D_LIB=build/ab/lib_$V.so; fi
      timeout -k 10 120 python tools/profile_scan.py $C 2>&1 | grep nrec >> $OUT/ab.log || exit 1
    done
  done
done
cat $OUT/ab.log
