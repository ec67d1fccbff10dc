#!/bin/bash
# hardware queues per process (GPU_MAX_HW_QUEUES) 8 vs 16 for the bench (main loop and config-3 overlapped passes)
set -o pipefail
OUT=gpurun_out/r03zb
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for Q in 8 16; do
    echo -n "queues $Q: " >> $OUT/q.log
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); h=d['roofline_hbm']; print('%.4g windows/s  cfg3 ovl fst %s  t2d %s' % (d['value'], ['%.4f' % x for x in h['overlapped']['pipeline_ms_reps']], ['%.4f' % x for x in h['t2d_t1d_overlapped']['pipeline_ms_reps']]))" >> $OUT/q.log || exit 1
  done
done
cat $OUT/q.log
