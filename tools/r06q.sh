#!/bin/bash
# round 6: the driver's bench command, four fresh processes, with the timing events made before the settle
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "streams or fst_out or deterministic" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3 4; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06q/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f.split('/')[-1], 'ms %.4f single %.4f kprep_t %.4f scan_t %.4f samples %d nofst %.4f withfst %s c2 %.3g c4 %.3g c5 %s' % (d['ms_per_step'], r['single_stream_pass_ms'], r['k_prep_ms'], r['scan_ms'], r['timed_samples'], d['t2d_t1d_only']['ms_per_step'], ['%.4f' % x for x in d['t2d_t1d_only']['with_fst_ms_per_step_runs']], d['config2_weak']['value'], d['config4_sims']['value'], d.get('config5_snp_windows', {}).get('value')))
PY
