#!/bin/bash
# round 6: config 2 replayed as per-stream HIP graphs (16 runs per plan) over 2 / 3 / 4 / 6 streams;
# R06AD3_RUNS="S:K ..." (tag b): other stream counts S and graph sizes K (0: run_streams)
O=gpurun_out/r06ad3${R06AD3_TAG}; mkdir -p $O
RUNS=${R06AD3_RUNS:-"2:8 3:8 4:8 6:8"}
for i in 1 2; do
for SK in $RUNS; do
  S=${SK%%:*}; K=${SK##*:}; T=s${S}; [ "$K" != 8 ] && T=s${S}_k${K}
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-variants --streams $S --config2-graph $K > $O/bench_${T}_$i.json 2> $O/bench_${T}_$i.err || { tail -30 $O/bench_${T}_$i.err; exit 1; }
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06ad3%s/bench_s*.json' % __import__('os').environ.get('R06AD3_TAG',''))):
    d=json.loads(open(f).read().strip().splitlines()[-1]); c=d['config2_weak']
    print(f.split('/')[-1], 'c2 %.4e ms %.5f enq %.5f steps %d' % (c['value'], c['ms_per_step'], c['host_enqueue_ms_per_step'], c['steps']))
PY
