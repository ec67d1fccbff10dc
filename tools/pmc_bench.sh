#!/bin/bash
# HBM traffic of the bench command itself: two rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE), kernel
# trace only, each under its own time limit; then the config-3 stream (tools/profile_scan.py config3 fst).
# usage: bash tools/pmc_bench.sh <tag>      -> gpurun_out/<tag>/pmc_bench/{p3,p4}, pmc_cfg3/{p3,p4}
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT/pmc_bench $OUT/pmc_cfg3
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_bench/p3 -o pmc -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-variants --config2-steps 40 > $OUT/pmc_bench/p3.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_bench/p4 -o pmc -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-variants --config2-steps 40 > $OUT/pmc_bench/p4.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_cfg3/p3 -o pmc -- python3 tools/profile_scan.py config3 3 fst > $OUT/pmc_cfg3/p3.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_cfg3/p4 -o pmc -- python3 tools/profile_scan.py config3 3 fst > $OUT/pmc_cfg3/p4.log 2>&1
echo "pmc rc=$?"
