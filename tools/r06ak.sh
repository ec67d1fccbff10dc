#!/bin/bash
# config 5 on 4 streams replayed as per-stream HIP graphs vs 2 streams with run_streams (A/B, interleaved),
# after the new graph-replay test for its shape
set -o pipefail
O=gpurun_out/r06ak; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "graph_replay" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do for g in 8 0; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-config2 --no-variants --no-e2e --no-cpu-baseline --config5-graph $g > $O/bench_g${g}_$i.log 2>&1 || { tail -20 $O/bench_g${g}_$i.log; exit 1; }
  tail -1 $O/bench_g${g}_$i.log > $O/bench_g${g}_$i.json
  python -c "import json;d=json.load(open('$O/bench_g${g}_$i.json'));c=d['config5_snp_windows'];print('graph $g', round(c['ms_per_step'],5), '%.3e'%c['value'], c['kernels_ms']['timed_loop'], round(c['roofline']['frac'],4), '| c4 %.3e'%d['config4_sims']['value'], '| c3', round(d['ms_per_step'],4))"
done; done
