#!/bin/bash
# round 6: the driver's bench command (config 3 only) with the timed steps sampling both kernels (default) or
# the scan kernel only (SFS2D_BENCH_TK=4), and with k_prep tiles of 32k / 128k SNPs (SFS2D_TILE), interleaved
O=gpurun_out/r06t; mkdir -p $O
for i in 1 2; do
for V in base tk4 t32k t128k; do
  case $V in base) E="";; tk4) E="SFS2D_BENCH_TK=4";; t32k) E="SFS2D_TILE=32768";; t128k) E="SFS2D_TILE=131072";; esac
  env $E timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-config2 > $O/bench_${V}_$i.json 2> $O/bench_${V}_$i.err || { tail -30 $O/bench_${V}_$i.err; exit 1; }
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06t/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f.split('/')[-1], 'ms %.4f single %.4f kprep %.4f scan %.4f kprep_t %.4f scan_t %.4f samples %d nofst %.4f later %s 20+500 %.4f' % (d['ms_per_step'], r['single_stream_pass_ms'], r['k_prep_alone_ms'], r['scan_alone_ms'], r['k_prep_ms'], r['scan_ms'], r['timed_samples'], d['t2d_t1d_only']['ms_per_step'], ['%.4f' % x for x in d['t2d_t1d_only']['with_fst_ms_per_step_runs']], d['config3_20kb_500kb']['ms_per_step']))
PY
