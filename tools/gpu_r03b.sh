#!/bin/bash
# round 3: new GPU tests (T1D/T2D, dict likelihood_scan, world-2 sharded drivers, config 3 full size) + bench
set -o pipefail
OUT=gpurun_out/r03b
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sims_batch.py tests/test_dist_gpu.py tests/test_config3.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -5 $OUT/pytest_gpu.log
grep -E "PASS|FAIL" $OUT/pytest_gpu.log | grep -E "t12|dist|config3|dict" | head -40
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-600
