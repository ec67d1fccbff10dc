#!/bin/bash
# round 6: HIP-graph replay of config 2's run sequence (sfs2d_graph_*): the graph parity tests, then
# config 2 (3 plans on 3 streams, >= 400 passes) with run_streams (k=0) vs graphs of 2k runs per plan.
# First session: one graph with the streams as forked branches; R06AD_TAG=b: one graph per stream.
O=gpurun_out/r06ad${R06AD_TAG}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "graph_replay or run_streams" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2; do
for K in 0 1 4 16; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-variants --config2-graph $K > $O/bench_k${K}_$i.json 2> $O/bench_k${K}_$i.err || { tail -30 $O/bench_k${K}_$i.err; exit 1; }
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06ad%s/bench_k*.json' % __import__('os').environ.get('R06AD_TAG',''))):
    d=json.loads(open(f).read().strip().splitlines()[-1]); c=d['config2_weak']
    print(f.split('/')[-1], 'c2 %.4e ms %.5f enq %.5f steps %d | c3 ms %.4f' % (c['value'], c['ms_per_step'], c['host_enqueue_ms_per_step'], c['steps'], d['ms_per_step']))
PY
