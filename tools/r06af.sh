#!/bin/bash
# round 6 final build: rocprofv3 kernel trace + stats of the driver's bench command
O=gpurun_out/r06af; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/rocprof_bench.json 2> $O/rocprof_bench.err || { tail -20 $O/rocprof_bench.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
tail -c 300 $O/rocprof_bench.json
