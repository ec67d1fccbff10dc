#!/bin/bash
# the driver's short bench command (20 steps): default vs fused background tables (2 launches per pass,
# SFS2D_FUSED=1) vs threaded enqueue (SFS2D_ENQ_THREADS=1)
set -o pipefail
OUT=gpurun_out/r03z
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for V in default fused enq; do
    case $V in default) E="";; fused) E="SFS2D_FUSED=1";; enq) E="SFS2D_ENQ_THREADS=1";; esac
    echo -n "$V: " >> $OUT/drv.log
    env $E timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-hbm-stream --no-e2e 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g windows/s  %.2f us/step  host %.2f us/step  k3 %.2f / %.2f us' % (d['value'], d['ms_per_step']*1e3, d['host_enqueue_ms_per_step']*1e3, d['kernels_ms']['k_scan_w']*1e3, d['kernels_ms']['k_scan_w_untimed_pass']*1e3))" >> $OUT/drv.log || exit 1
    echo -n "$V 400: " >> $OUT/drv.log
    env $E timeout -k 10 200 python bench.py --no-cpu-baseline --no-hbm-stream --no-e2e 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4g windows/s  %.2f us/step  host %.2f us/step' % (d['value'], d['ms_per_step']*1e3, d['host_enqueue_ms_per_step']*1e3))" >> $OUT/drv.log || exit 1
  done
done
cat $OUT/drv.log
