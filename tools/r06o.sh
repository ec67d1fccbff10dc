#!/bin/bash
# round 6: the N > 1 bench path rehearsed on one GPU (every rank on GPU 0, gloo: a code-path check, not a
# measurement), then one rank's config-3 share at N = 1 / 2 / 4 / 8 (32 / 16 / 8 / 4 chromosomes) timed alone
O=gpurun_out/r06o; mkdir -p $O
SFS2D_BENCH_SHARED_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --no-config2 --no-variants > $O/bench_n2.log 2>&1 || { tail -30 $O/bench_n2.log; exit 1; }
tail -1 $O/bench_n2.log > $O/bench_n2.json
for C in 32 16 8 4; do
  timeout -k 10 200 python tools/exp_streams_cfg3.py 40 fst 1 $C >> $O/share.txt 2>> $O/share.err || { tail -20 $O/share.err; exit 1; }
done
cat $O/share.txt
python3 -c "
import json; d=json.loads(open('$O/bench_n2.json').read()); print({k: d.get(k) for k in ('value','ms_per_step','n_gpus','gather_ms','gather_ms_per_step','gathered','shared_gpu_rehearsal')})"
