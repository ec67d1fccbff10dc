#!/bin/bash
# Repeatability of the streams x hardware-queue settings (config 2, bench.py 400 steps and the
# driver's 20 steps).   usage: bash tools/streams_probe3.sh <tag>
set -o pipefail
TAG=${1:-streams3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --no-hbm-stream $BARGS > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  tail -1 $OUT/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$name', round(d['value']/1e6,1), 'M windows/s', round(d['ms_per_step']*1e3,2), 'us/step', 'k3', round(k['k_scan_w']*1e3,2))"
}
for r in 1 2 3; do
  BARGS="--streams 3" run s3_q8_$r GPU_MAX_HW_QUEUES=8
  BARGS="--streams 2" run s2_q8_$r GPU_MAX_HW_QUEUES=8
  BARGS="--streams 3 --steps 20 --warmup 5" run s3_q8_drv_$r GPU_MAX_HW_QUEUES=8
  BARGS="--streams 2 --steps 20 --warmup 5" run s2_q4_drv_$r GPU_MAX_HW_QUEUES=4
done
BARGS="--streams 3" run s3_q6 GPU_MAX_HW_QUEUES=6
BARGS="--streams 3" run s3_q4 GPU_MAX_HW_QUEUES=4
