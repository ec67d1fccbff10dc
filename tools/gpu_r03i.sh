#!/bin/bash
# k_prep Fst terms: alt-count table (default) vs conversions (SFS2D_EXP_FST_NOTB)
set -o pipefail
OUT=gpurun_out/r03i
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for V in NONE SFS2D_EXP_FST_NOTB; do
    echo -n "$V " >> $OUT/ab.log
    SFS2D_LIB=build/ab/lib_$V.so timeout -k 10 120 python tools/profile_scan.py config3 30 fst 2>&1 | grep nrec >> $OUT/ab.log || exit 1
  done
done
cat $OUT/ab.log
