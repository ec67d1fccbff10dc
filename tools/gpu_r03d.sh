#!/bin/bash
# A/B: k_prep waves-per-EU hint (0 = none: 87 VGPRs for the Fst variant; 6; 8 = 64 VGPRs)
set -o pipefail
OUT=gpurun_out/r03d
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for W in 0 6 8; do
    for c in config2 config3; do
      for f in fst nofst; do
        echo -n "wpe$W $f " >> $OUT/ab.log
        SFS2D_LIB=build/ab/lib_wpe$W.so timeout -k 10 120 python tools/profile_scan.py $c 30 $f 2>&1 | grep nrec >> $OUT/ab.log || exit 1
      done
    done
  done
done
cat $OUT/ab.log
