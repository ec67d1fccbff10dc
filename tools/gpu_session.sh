#!/bin/bash
# One GPU session: parity tests, config timings (with Fst), bench, rocprofv3 kernel-trace of the bench.
# usage: bash tools/gpu_session.sh <tag> [skip-tests]
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
for c in config2 config3 config5; do
  timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> $OUT/profile_scan.log 2>&1 || { cat $OUT/profile_scan.log; exit 1; }
done
cat $OUT/profile_scan.log
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline > $OUT/rocprof_bench.log 2>&1 || { tail -20 $OUT/rocprof_bench.log; exit 1; }
find $OUT/prof -name "*stats*"
