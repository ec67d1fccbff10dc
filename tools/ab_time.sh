#!/bin/bash
# Interleaved kernel timings (HIP events, tools/profile_scan.py) of several library builds.
# usage: bash tools/ab_time.sh <rounds> <lib.so> [lib.so ...]
set -o pipefail
R=$1; shift
for r in $(seq 1 $R); do
  for L in "$@"; do
    for c in config2 config3; do
      echo -n "$(basename $L) "
      SFS2D_LIB=$L timeout -k 10 120 python tools/profile_scan.py $c 50 fst 2>&1 | grep nrec || exit 1
    done
  done
done
