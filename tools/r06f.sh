#!/bin/bash
# round 6: k_prep's slot-search blocks (SFS2D_SEG=prepsearch) vs k_prep's segmentation, config 3, interleaved
O=gpurun_out/r06f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "records_per_chrom or fst_vs_oracle or config2 or scan_kernels_agree" > $O/pytest_default.log 2>&1 || { tail -30 $O/pytest_default.log; exit 1; }
SFS2D_SEG=prepsearch timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "records_per_chrom or fst_vs_oracle or config2 or scan_kernels_agree" > $O/pytest_ps.log 2>&1 || { tail -30 $O/pytest_ps.log; exit 1; }
for i in 1 2; do
for S in prep prepsearch; do
  SFS2D_SEG=$S timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims > $O/bench_${S}_$i.json 2> $O/bench_${S}_$i.err || { tail -30 $O/bench_${S}_$i.err; exit 1; }
done; done
tail -2 $O/pytest_default.log $O/pytest_ps.log
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06f/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f, 'ms %.4f single %.4f kprep %.4f scan %.4f kprep_t %.4f scan_t %.4f nofst %.4f c2 %.3g' % (d['ms_per_step'], r['single_stream_pass_ms'], r['k_prep_alone_ms'], r['scan_alone_ms'], r['k_prep_ms'], r['scan_ms'], d['t2d_t1d_only']['ms_per_step'], d['config2_weak']['value']))
PY
