#!/bin/bash
# round 6 final check: the GPU suite, smoke, the default bench line and the driver's command (twice)
O=gpurun_out/r06ae; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
for i in 1 2; do
  timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$i.json 2> $O/bench_driver_$i.err || { tail -30 $O/bench_driver_$i.err; exit 1; }
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06ae/bench*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], 'value %.4e ms %.4f frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac']),
          'c2 %.4e' % d['config2_weak']['value'], 'c4 %.4e' % d['config4_sims']['value'], 'c5 %.4e' % d['config5_snp_windows']['value'],
          'cpu %.4e' % d['cpu_baseline']['value'])
PY
