#!/bin/bash
# round 6: HIP-graph replay with config 2's runs on ONE stream (--streams 1): is the graph's slowness the
# multi-stream branches or the per-node launches?
O=gpurun_out/r06ad2; mkdir -p $O
for K in 0 8; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-variants --streams 1 --config2-graph $K > $O/bench_s1_k${K}.json 2> $O/bench_s1_k${K}.err || { tail -30 $O/bench_s1_k${K}.err; exit 1; }
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06ad2/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); c=d['config2_weak']
    print(f.split('/')[-1], 'c2 %.4e ms %.5f enq %.5f steps %d' % (c['value'], c['ms_per_step'], c['host_enqueue_ms_per_step'], c['steps']))
PY
