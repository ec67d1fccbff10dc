#!/bin/bash
# round 6: k_prep's segmentation over compact positions (2 B per SNP) -- parity, then k_prep / scan times and
# the bench with (default) and without them (SFS2D_POS16=0), interleaved
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_config3.py tests/test_dist_gpu.py tests/test_multires.py -x -q --timeout 300 --timeout-method thread -k "compact or joint or records_per_chrom or called_counts or config3 or fst_vs_oracle or scan_kernels_agree or sparse or split or multires or attach" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for i in 1 2; do
for V in 1 0; do
  SFS2D_POS16=$V timeout -k 10 120 python tools/ktime.py fst 7 | sed "s/^/POS16=$V /" >> $O/ktime.txt 2>> $O/ktime.err || { tail -20 $O/ktime.err; exit 1; }
done; done
cat $O/ktime.txt
for i in 1 2; do
for V in 1 0; do
  SFS2D_POS16=$V timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims > $O/bench_pos16_${V}_$i.json 2> $O/bench_pos16_${V}_$i.err || { tail -30 $O/bench_pos16_${V}_$i.err; exit 1; }
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06j/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f.split('/')[-1], 'ms %.4f single %.4f kprep %.4f scan %.4f kprep_t %.4f scan_t %.4f nofst %.4f c2 %.3g 500kb %.4f' % (d['ms_per_step'], r['single_stream_pass_ms'], r['k_prep_alone_ms'], r['scan_alone_ms'], r['k_prep_ms'], r['scan_ms'], d['t2d_t1d_only']['ms_per_step'], d['config2_weak']['value'], d['config3_20kb_500kb']['ms_per_step']))
PY
