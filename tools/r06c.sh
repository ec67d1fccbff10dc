#!/bin/bash
# round 6: the driver's bench command at N = 1 (configs 2-5 keys) and the N = 2 shared-GPU rehearsal of
# the per-pass gathered loop
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench_driver_cmd.err || { tail -30 $O/bench_driver_cmd.err; exit 1; }
SFS2D_BENCH_SHARED_GPU=1 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-config2 > $O/bench_shared_n2.json 2> $O/bench_shared_n2.err || { tail -30 $O/bench_shared_n2.err; exit 1; }
echo done
