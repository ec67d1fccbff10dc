#!/bin/bash
# round 6: k_scan_w's batch's last window prefetching too, the finish running with the next rows in flight (pfx)
# vs the default: parity subset, kernel times, config-3 bench
O=gpurun_out/r06u; mkdir -p $O
V=2dsfs-scan_amd/csrc/variants
SFS2D_LIB=$V/libsfs2d_pfx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_config3.py -x -q --timeout 300 --timeout-method thread -k "records_per_chrom or fst_vs_oracle or scan_kernels_agree or joint or dropin_class or config3 or streams or config2 or zero or exact" > $O/pytest_pfx.log 2>&1 || { tail -30 $O/pytest_pfx.log; exit 1; }
tail -1 $O/pytest_pfx.log
for i in 1 2; do
for L in 2dsfs-scan_amd/csrc/libsfs2d.so $V/libsfs2d_pfx.so; do
  SFS2D_LIB=$L timeout -k 10 120 python tools/ktime.py fst 7 >> $O/ktime.txt 2>> $O/ktime.err || { tail -20 $O/ktime.err; exit 1; }
done; done
cat $O/ktime.txt
for i in 1 2; do
for L in 2dsfs-scan_amd/csrc/libsfs2d.so $V/libsfs2d_pfx.so; do
  n=$(basename $L .so)
  SFS2D_LIB=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims > $O/bench_${n}_$i.json 2> $O/bench_${n}_$i.err || { tail -30 $O/bench_${n}_$i.err; exit 1; }
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06u/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f.split('/')[-1], 'ms %.4f single %.4f kprep %.4f scan %.4f kprep_t %.4f scan_t %.4f nofst %.4f c2 %.3g 20+500 %.4f' % (d['ms_per_step'], r['single_stream_pass_ms'], r['k_prep_alone_ms'], r['scan_alone_ms'], r['k_prep_ms'], r['scan_ms'], d['t2d_t1d_only']['ms_per_step'], d['config2_weak']['value'], d['config3_20kb_500kb']['ms_per_step']))
PY
