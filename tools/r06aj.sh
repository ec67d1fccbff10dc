#!/bin/bash
# the driver's bench command four times (fresh processes) with dense_kernel_samples as 10 repeated timed-loop-like loops
set -o pipefail
O=gpurun_out/r06aj; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.log 2>&1 || { tail -20 $O/bench_driver_$i.log; exit 1; }
  tail -1 $O/bench_driver_$i.log > $O/bench_driver_$i.json
  python -c "import json;d=json.load(open('$O/bench_driver_$i.json'));r=d['roofline'];print($i, round(d['ms_per_step'],4), round(r['ms'],4), r['dense_check']['ms'], r['dense_check']['launches'])"
done
