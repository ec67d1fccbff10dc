#!/bin/bash
# overlapped passes with the scan kernel capped per CU: config 2 / config 3, Fst on and off
set -o pipefail
OUT=gpurun_out/r03h
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 200 python tools/exp_streams.py config2 400 fst "1,0 2,0 3,0 2,1 3,1 4,1 3,2 4,2 6,1" >> $OUT/streams.log 2>&1 &&
timeout -k 10 200 python tools/exp_streams.py config3 24 fst "1,0 2,0 2,1 3,1 1,0 2,1" >> $OUT/streams.log 2>&1 &&
timeout -k 10 200 python tools/exp_streams.py config3 24 nofst "1,0 2,1 3,1" >> $OUT/streams.log 2>&1
cat $OUT/streams.log
