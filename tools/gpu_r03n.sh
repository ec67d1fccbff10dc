#!/bin/bash
# Round-3 profiles: rocprofv3 kernel trace + stats of the bench, HBM bytes (FETCH/WRITE passes) of the
# bench and of the config-3 stream, SQ counters of the config-3 stream (k_scan_w LDS conflicts)
set -o pipefail
TAG=${1:-r03n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline > $OUT/rocprof_bench.log 2>&1 || { tail -20 $OUT/rocprof_bench.log; exit 1; }
tail -1 $OUT/rocprof_bench.log | cut -c1-300
bash tools/pmc_bench.sh $TAG || exit 1
bash tools/pmc_k3.sh $TAG config3 fst || exit 1
find $OUT -name "*stats*.csv" | head
