#!/bin/bash
# round 6: the driver's bench command (config 3 only), run_streams as built vs SFS2D_CHAIN=2 (the first 2 x plans runs' k_preps chained
# one after another, then free), eight fresh processes each, interleaved
O=gpurun_out/r06x; mkdir -p $O
for i in 1 2 3 4 5 6 7 8; do
for C in none 2; do
  if [ $C = none ]; then unset SFS2D_CHAIN; else export SFS2D_CHAIN=$C; fi
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-config2 > $O/bench_c${C}_$i.json 2> $O/bench_c${C}_$i.err || { tail -30 $O/bench_c${C}_$i.err; exit 1; }
done; done
unset SFS2D_CHAIN
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06x/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f.split('/')[-1], 'ms %.4f single %.4f kprep_t %.4f scan_t %.4f nofst %.4f later %s 20+500 %.4f' % (d['ms_per_step'], r['single_stream_pass_ms'], r['k_prep_ms'], r['scan_ms'], d['t2d_t1d_only']['ms_per_step'], ['%.4f' % x for x in d['t2d_t1d_only']['with_fst_ms_per_step_runs']], d['config3_20kb_500kb']['ms_per_step']))
PY
