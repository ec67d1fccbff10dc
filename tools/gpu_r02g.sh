#!/bin/bash
# Round-2 final GPU session: full parity suite + kernel timings + bench + rocprofv3 kernel trace,
# PMC FETCH/WRITE passes, the driver's 20-step command twice.   usage: bash tools/gpu_r02g.sh <tag>
set -o pipefail
TAG=${1:-r02g}
bash tools/gpu_session.sh $TAG &&
bash tools/pmc_bench.sh $TAG &&
for r in 1 2; do
  timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver_$r.log 2>&1 || exit 1
  tail -1 gpurun_out/$TAG/bench_driver_$r.log
done
