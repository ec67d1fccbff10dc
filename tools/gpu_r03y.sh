#!/bin/bash
# why bench.py's config-3 overlapped passes read slower than tools/exp_streams_cfg3.py (tools/hbm_probe.py)
set -o pipefail
OUT=gpurun_out/r03y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python tools/hbm_probe.py > $OUT/probe_alone.log 2>&1 || { tail -20 $OUT/probe_alone.log; exit 1; }
timeout -k 10 200 python tools/hbm_probe.py with-loop > $OUT/probe_loop.log 2>&1 || { tail -20 $OUT/probe_loop.log; exit 1; }
timeout -k 10 200 python tools/exp_streams_cfg3.py 24 nofst 1 > $OUT/exp.log 2>&1 || { tail -20 $OUT/exp.log; exit 1; }
grep -v amdgpu.ids $OUT/probe_alone.log $OUT/probe_loop.log $OUT/exp.log
bash tools/gpu_r03z.sh
