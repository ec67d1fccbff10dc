#!/bin/bash
# Native N>1 step loop on one rank (bench.py --dist-loop) with 1 and 2 streams (one RCCL
# communicator per stream), and the driver's 20-step command with 2 streams.
# usage: bash tools/streams_dist_probe.sh <tag>
set -o pipefail
TAG=${1:-streams_dist}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_dist_native.py tests/test_gpu_parity.py -k "streams or scan_gather" -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for s in 1 2; do
  timeout -k 10 240 python bench.py --dist-loop --streams $s --no-cpu-baseline --no-hbm-stream > $OUT/dist_s$s.log 2>&1 || { tail -20 $OUT/dist_s$s.log; exit 1; }
  tail -1 $OUT/dist_s$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('dist-loop streams $s', round(d['value']/1e6,1), 'M windows/s', round(d['ms_per_step']*1e3,2), 'us/step', d['config']['parallelism'], d.get('dist_step_ms_by_placement'))"
done
for r in 1 2; do
  timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-hbm-stream > $OUT/driver_s2_$r.log 2>&1 || { tail -20 $OUT/driver_s2_$r.log; exit 1; }
  tail -1 $OUT/driver_s2_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('driver cmd streams 2', round(d['value']/1e6,1), 'M windows/s', round(d['ms_per_step']*1e3,2), 'us/step')"
done
