#!/bin/bash
# the bench line with config 3's overlapped passes as its pipeline entry (median of 3 repetitions)
set -o pipefail
OUT=gpurun_out/r03za
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
