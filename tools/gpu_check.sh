#!/bin/bash
# One GPU session: parity tests, per-config kernel timings, stamps, bench, rocprof kernel trace.
# usage: bash tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
for c in config2 config3 config5; do
  timeout -k 10 180 python tools/profile_scan.py $c 10 >> $OUT/profile_scan.log 2>&1 || { cat $OUT/profile_scan.log; exit 1; }
done
cat $OUT/profile_scan.log
for c in config2 config3; do
  SFS2D_LIB=2dsfs-scan_amd/csrc/libsfs2d_stamps.so timeout -k 10 180 python tools/stamps.py $c >> $OUT/stamps.log 2>&1 || { cat $OUT/stamps.log; exit 1; }
done
cat $OUT/stamps.log
timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
cat $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline > $OUT/rocprof_bench.log 2>&1 || { tail -20 $OUT/rocprof_bench.log; exit 1; }
find $OUT/prof -name "*stats*" | head
