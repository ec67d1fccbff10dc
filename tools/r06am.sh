#!/bin/bash
# round 6 final check: full GPU suite (with the config-5-shape graph-replay test), smoke, the driver's bench command
set -o pipefail
O=gpurun_out/r06am; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log > $O/bench_driver.json
python -c "import json;d=json.load(open('$O/bench_driver.json'));r=d['roofline'];print(round(d['ms_per_step'],4), '%.3e'%d['value'], round(r['frac'],4), r['dense_check']['ms'])"
