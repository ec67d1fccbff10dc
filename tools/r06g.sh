#!/bin/bash
# round 6: where k_scan_w's per-window time goes (ablation builds: 256 no per-window wave sums, 520 no
# batched finish, 808 neither + no 1D end pass) and the slot-clear-free Fst build (noclr), config 3
O=gpurun_out/r06g; mkdir -p $O
V=2dsfs-scan_amd/csrc/variants
export SFS2D_ALLOW_ABLATION=1
for i in 1 2; do
for L in 2dsfs-scan_amd/csrc/libsfs2d.so $V/libsfs2d_abl256.so $V/libsfs2d_abl520.so $V/libsfs2d_abl808.so $V/libsfs2d_noclr.so; do
  SFS2D_LIB=$L timeout -k 10 120 python tools/ktime.py fst 7 >> $O/ktime.txt 2>> $O/ktime.err || { tail -20 $O/ktime.err; exit 1; }
done; done
cat $O/ktime.txt
for i in 1 2; do
for L in 2dsfs-scan_amd/csrc/libsfs2d.so $V/libsfs2d_noclr.so; do
  n=$(basename $L .so)
  SFS2D_LIB=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-sims --no-config2 > $O/bench_${n}_$i.json 2> $O/bench_${n}_$i.err || { tail -30 $O/bench_${n}_$i.err; exit 1; }
done; done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r06g/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1]); r=d['rank0']
    print(f, 'ms %.4f single %.4f kprep %.4f scan %.4f kprep_t %.4f scan_t %.4f nofst %.4f' % (d['ms_per_step'], r['single_stream_pass_ms'], r['k_prep_alone_ms'], r['scan_alone_ms'], r['k_prep_ms'], r['scan_ms'], d['t2d_t1d_only']['ms_per_step']))
PY
