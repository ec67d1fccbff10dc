#!/bin/bash
# round 6: k_slots_search for per-chromosome plans (counts-only k_prep) -- full GPU suite, then the bench
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
SFS2D_SEG=prep timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-config2 > $O/bench_prep.json 2> $O/bench_prep.err || { tail -30 $O/bench_prep.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-config2 > $O/bench2.json 2> $O/bench2.err || { tail -30 $O/bench2.err; exit 1; }
echo done
