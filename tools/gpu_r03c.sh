#!/bin/bash
# round 3: counts plans -- bins vs counts timings (with / without Fst), then the full-size config-3 and world-2 tests
set -o pipefail
OUT=gpurun_out/r03c
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
for c in config2 config3; do
  for m in 0 1; do
    echo "SFS2D_CNT=$m" >> $OUT/profile_scan.log
    SFS2D_CNT=$m timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> $OUT/profile_scan.log 2>&1 || { cat $OUT/profile_scan.log; exit 1; }
    SFS2D_CNT=$m timeout -k 10 180 python tools/profile_scan.py $c 20 >> $OUT/profile_scan.log 2>&1 || { cat $OUT/profile_scan.log; exit 1; }
  done
done
cat $OUT/profile_scan.log
timeout -k 10 500 python -u -m pytest tests/test_config3.py tests/test_dist_gpu.py -m gpu -x -v -s --timeout 450 --timeout-method thread > $OUT/pytest_big.log 2>&1 || { tail -60 $OUT/pytest_big.log; exit 1; }
tail -5 $OUT/pytest_big.log
