#!/bin/bash
# Config-2 overlapped-pass throughput vs scan workgroup count (SFS2D_WGS) and k_prep tile
# (SFS2D_TILE), 3 streams, bench.py 400 steps.   usage: bash tools/overlap_sweep.sh <tag>
set -o pipefail
TAG=${1:-ovsweep}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --no-hbm-stream $BARGS > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; exit 1; }
  tail -1 $OUT/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels_ms']; print('$name', round(d['value']/1e6,1), 'M windows/s', round(d['ms_per_step']*1e3,2), 'us/step; k1/k2/k3 iso', round(k['k_prep']*1e3,2), round(k['k_bg_slice']*1e3,2), round(d['roofline']['ms']*1e3,2))"
}
run base1
run wgs128 SFS2D_WGS=128
run wgs192 SFS2D_WGS=192
run wgs256 SFS2D_WGS=256
run tile8k SFS2D_TILE=8192
run tile16k SFS2D_TILE=16384
run base2
run wgs192_t8k SFS2D_WGS=192 SFS2D_TILE=8192
