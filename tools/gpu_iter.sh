#!/bin/bash
# Iteration check: parity tests, config timings (Fst on), stamps.  usage: bash tools/gpu_iter.sh <tag>
set -o pipefail
TAG=${1:-it}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for c in config2 config3 config5; do
  timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> $OUT/profile_scan.log 2>&1 || { cat $OUT/profile_scan.log; exit 1; }
done
cat $OUT/profile_scan.log
for c in config2 config3; do
  SFS2D_LIB=2dsfs-scan_amd/csrc/libsfs2d_stamps.so timeout -k 10 180 python tools/stamps.py $c >> $OUT/stamps.log 2>&1 || { cat $OUT/stamps.log; exit 1; }
done
grep -v "^ *[0-9]" $OUT/stamps.log | head -20
