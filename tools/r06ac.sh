#!/bin/bash
# round 6: how often the first timed loop of the driver's bench command (config 3 only, 20 steps) lands in
# the slow phase, by how densely its passes carry kernel events (SFS2D_BENCH_EVERY, per plan).
#   R06AC_E="d 1"  : every 2nd pass (the old default at 20 steps) vs every pass
#   R06AC_E="4 10" : every 4th / 10th pass
#   R06AC_E="n"    : the new default (2 sampled passes per plan: first + middle; session d: first + last), then one full default bench line
O=gpurun_out/r06ac${R06AC_TAG}; mkdir -p $O
for i in 1 2 3 4 5 6 7 8; do
for E in $R06AC_E; do
  if [ $E = d ] || [ $E = n ]; then unset SFS2D_BENCH_EVERY; else export SFS2D_BENCH_EVERY=$E; fi
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-config2 > $O/bench_e${E}_$i.json 2> $O/bench_e${E}_$i.err || { tail -30 $O/bench_e${E}_$i.err; exit 1; }
done; done
unset SFS2D_BENCH_EVERY
if [ "$R06AC_E" = n ]; then
  timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -30 $O/bench_full.err; exit 1; }
  tail -c 600 $O/bench_full.json; echo
fi
python3 - <<'PY'
import json,glob,os
for f in sorted(glob.glob('gpurun_out/r06ac%s/bench_e*.json' % os.environ.get('R06AC_TAG',''))):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f.split('/')[-1], 'ms %.4f kprep_t %.4f scan_t %.4f samples %d later %s' % (d['ms_per_step'], r['k_prep_ms'], r['scan_ms'], r['timed_samples'], ['%.4f' % x for x in d['t2d_t1d_only']['with_fst_ms_per_step_runs']]))
PY
