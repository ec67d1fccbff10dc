#!/bin/bash
# One GPU call, as a list of steps, each under its own time limit; the first failing step ends the call.
# usage: bash tools/gpu.sh <tag> <step>...      outputs under gpurun_out/<tag>/
#   tests[=<pytest -k expr>]  the -m gpu suite       smoke    __graft_entry__.smoke()
#   bench                     python bench.py         driver   the driver's bench command (20 steps)
#   rocprof                   rocprofv3 kernel trace + stats of the bench
#   pmc                       HBM bytes of the bench and config 3 (tools/pmc_bench.sh)
#   sq3                       SQ / byte counter passes over config 3 with Fst (tools/pmc_k3.sh)
#   profile                   per-kernel times of configs 2 / 3 / 5 (tools/profile_scan.py)
set -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests|tests=*)
      K=${step#tests}; K=${K#=}
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread ${K:+-k "$K"} \
        > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
      tail -3 $OUT/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
      tail -1 $OUT/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -30 $OUT/bench.log; exit 1; }
      tail -1 $OUT/bench.log | cut -c1-600 ;;
    driver)
      timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -30 $OUT/bench_driver.log; exit 1; }
      tail -1 $OUT/bench_driver.log | cut -c1-600 ;;
    rocprof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e \
        > $OUT/rocprof_bench.log 2>&1 || { tail -20 $OUT/rocprof_bench.log; exit 1; }
      find $OUT/prof -name "*stats*" ;;
    pmc) bash tools/pmc_bench.sh $TAG || exit 1 ;;
    sq3) bash tools/pmc_k3.sh $TAG config3 fst || exit 1 ;;
    profile)
      for c in config2 config3 config5; do
        timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> $OUT/profile_scan.log 2>&1 || { cat $OUT/profile_scan.log; exit 1; }
      done
      cat $OUT/profile_scan.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu.sh $TAG: done"
