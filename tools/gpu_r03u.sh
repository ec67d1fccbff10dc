#!/bin/bash
# k_scan_w variants: pipelined row pairs (PIPE), next-window rows prefetched after the sums (LPF), both;
# parity subset on PIPE, then interleaved timings against the tree's build
set -o pipefail
OUT=gpurun_out/r03u
mkdir -p $OUT
export TMPDIR=/tmp
SFS2D_LIB=build/ab/lib_PIPE.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "parity or fst or multires or config" > $OUT/tests_pipe.log 2>&1 || { tail -30 $OUT/tests_pipe.log; exit 1; }
tail -1 $OUT/tests_pipe.log
for r in 1 2; do
  for L in 2dsfs-scan_amd/csrc/libsfs2d.so build/ab/lib_LPF.so build/ab/lib_PIPE.so build/ab/lib_PIPELPF.so; do
    for C in "config3 30 fst" "config3 30" "config2 30 fst"; do
      echo -n "$(basename $L) $C: " >> $OUT/ab.log
      SFS2D_LIB=$L timeout -k 10 120 python tools/profile_scan.py $C 2>&1 | grep nrec >> $OUT/ab.log || exit 1
    done
  done
done
cat $OUT/ab.log
