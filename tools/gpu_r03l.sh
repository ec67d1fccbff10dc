#!/bin/bash
# config 3 with Fst: overlapped passes (S streams, scan capped at W workgroups per CU) with Fst summed
# in the scan (SFS2D_FST_SCAN=1, k_prep Fst-free and bandwidth-bound) vs k_prep's sums
set -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
SFS2D_FST_SCAN=1 timeout -k 10 200 python tools/exp_streams.py config3 24 fst "1,0 2,0 2,1 3,1 2,2 3,2" 2>&1 | sed 's/^/FST_SCAN=1 /' >> $OUT/streams.log &&
SFS2D_FST_SCAN=0 timeout -k 10 200 python tools/exp_streams.py config3 24 fst "1,0 2,1 3,1" 2>&1 | sed 's/^/FST_SCAN=0 /' >> $OUT/streams.log &&
SFS2D_FST_SCAN=1 timeout -k 10 200 python tools/exp_streams.py config2 400 fst "1,0 2,0 3,0 3,1" 2>&1 | sed 's/^/FST_SCAN=1 /' >> $OUT/streams.log
cat $OUT/streams.log
