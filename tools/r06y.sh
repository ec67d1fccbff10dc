#!/bin/bash
# round 6 measurement session (the final round-6 build: joint histogram, ln prefetch, LDS ln table): full GPU suite, smoke, bench (default and the
# driver's command), rocprofv3 kernel trace of the driver's command, PMC bytes of the bench command
# (FETCH_SIZE / WRITE_SIZE passes) and k_scan_w's SQ counters on config 3
set -o pipefail
O=gpurun_out/r06y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log > $O/bench_driver.json
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver2.log 2>&1 || { tail -20 $O/bench_driver2.log; exit 1; }
tail -1 $O/bench_driver2.log > $O/bench_driver2.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/rocprof_bench.log 2>&1 || { tail -20 $O/rocprof_bench.log; exit 1; }
mkdir -p $O/pmc_bench
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_bench/p3 -o pmc -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-variants --no-sims --config2-steps 40 > $O/pmc_bench/p3.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_bench/p4 -o pmc -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-variants --no-sims --config2-steps 40 > $O/pmc_bench/p4.log 2>&1 || { echo "pmc bench failed"; tail -5 $O/pmc_bench/*.log; exit 1; }
bash tools/pmc_k3.sh r06y config3 fst
echo done
