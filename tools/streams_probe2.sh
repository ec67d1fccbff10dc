#!/bin/bash
# Streams x hardware queues x background path probe (config 2, bench.py 400 steps).
# usage: bash tools/streams_probe2.sh <tag>
set -o pipefail
TAG=${1:-streams2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {   # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --no-hbm-stream $BARGS > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  tail -1 $OUT/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$name', round(d['value']/1e6,1), 'M windows/s', round(d['ms_per_step']*1e3,2), 'us/step', 'k3', round(k['k_scan_w']*1e3,2))"
}
BARGS="--streams 2" run s2_q4 GPU_MAX_HW_QUEUES=4
BARGS="--streams 3" run s3_q8 GPU_MAX_HW_QUEUES=8
BARGS="--streams 4" run s4_q8 GPU_MAX_HW_QUEUES=8
BARGS="--streams 6" run s6_q8 GPU_MAX_HW_QUEUES=8
BARGS="--streams 2" run s2_fused SFS2D_FUSED=1
BARGS="--streams 4" run s4_fused_q8 SFS2D_FUSED=1 GPU_MAX_HW_QUEUES=8
