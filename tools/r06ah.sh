#!/bin/bash
# round 6, final session (container rebuilt from HEAD): full GPU suite, smoke, bench (default and the
# driver's command twice, with the dense kernel-sample cross-check), rocprofv3 kernel trace of the driver's command
set -o pipefail
O=gpurun_out/r06ah; mkdir -p $O
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
echo done
