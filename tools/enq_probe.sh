#!/bin/bash
# Threaded vs single-thread enqueue of the overlapped passes (bench.py, config 2), after the GPU suite.
# usage: bash tools/enq_probe.sh <tag>
set -o pipefail
TAG=${1:-enq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --no-hbm-stream $BARGS > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  tail -1 $OUT/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$name', round(d['value']/1e6,1), 'M windows/s', round(d['ms_per_step']*1e3,2), 'us/step; host enqueue', round(d['host_enqueue_ms_per_step']*1e3,2), 'us/step; k3', round(k['k_scan_w']*1e3,2), round(d['roofline']['ms']*1e3,2))"
}
BARGS="" run thr_1 SFS2D_ENQ_THREADS=1
BARGS="" run one_1 SFS2D_ENQ_THREADS=0
BARGS="" run thr_2 SFS2D_ENQ_THREADS=1
BARGS="" run one_2 SFS2D_ENQ_THREADS=0
BARGS="--streams 4" run thr_s4 SFS2D_ENQ_THREADS=1
BARGS="--streams 2" run thr_s2 SFS2D_ENQ_THREADS=1
BARGS="--steps 20 --warmup 5" run thr_drv_1 SFS2D_ENQ_THREADS=1
BARGS="--steps 20 --warmup 5" run one_drv_1 SFS2D_ENQ_THREADS=0
BARGS="--steps 20 --warmup 5" run thr_drv_2 SFS2D_ENQ_THREADS=1
BARGS="--steps 20 --warmup 5" run one_drv_2 SFS2D_ENQ_THREADS=0
