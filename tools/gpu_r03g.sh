#!/bin/bash
# PMC passes on config 3 (counts plans; with and without Fst) + K1/K2 overlap with fewer scan workgroups
set -o pipefail
OUT=gpurun_out/r03g
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
bash tools/pmc_k3.sh r03g config3 fst > $OUT/pmc_fst.log 2>&1 && bash tools/pmc_k3.sh r03g config3 > $OUT/pmc_nofst.log 2>&1 || { cat $OUT/pmc_*.log; exit 1; }
for W in 256 384; do
  echo "SFS2D_WGS=$W" >> $OUT/streams.log
  SFS2D_WGS=$W timeout -k 10 200 python tools/exp_streams_cfg3.py 24 >> $OUT/streams.log 2>&1 || { cat $OUT/streams.log; exit 1; }
done
cat $OUT/streams.log
