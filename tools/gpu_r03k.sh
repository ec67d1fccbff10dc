#!/bin/bash
# Fst in k_scan_w (fst_scan) vs k_prep's sums / k_bg_slice's Fst workgroups (SFS2D_FST_SCAN=0):
# Fst parity tests, then config 3 / config 2 timings
set -o pipefail
OUT=gpurun_out/r03k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_multires.py -k "fst or Fst or multires or attach or streams" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  for V in 1 0; do
    for C in config3 config2; do
      echo -n "FST_SCAN=$V $C " >> $OUT/ab.log
      SFS2D_FST_SCAN=$V timeout -k 10 120 python tools/profile_scan.py $C 30 fst 2>&1 | grep nrec >> $OUT/ab.log || exit 1
    done
  done
done
cat $OUT/ab.log
