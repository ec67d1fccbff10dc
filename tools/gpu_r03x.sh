#!/bin/bash
# round-3 final profile set on the tree's build: full GPU suite, smoke, bench, rocprofv3 kernel trace of
# the bench, HBM bytes (FETCH_SIZE / WRITE_SIZE passes) of the bench and config 3, SQ counters of config 3
set -o pipefail
OUT=gpurun_out/r03x
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=8   # bench.py raises it in-process, too late under rocprofv3 (its library starts HIP first)
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.log 2>&1 || { tail -20 $OUT/bench_driver.log; exit 1; }
tail -1 $OUT/bench_driver.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e > $OUT/rocprof_bench.log 2>&1 || { tail -20 $OUT/rocprof_bench.log; exit 1; }
bash tools/pmc_bench.sh r03x || exit 1
bash tools/pmc_k3.sh r03x config3 fst || exit 1
echo done
