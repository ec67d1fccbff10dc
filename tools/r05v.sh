set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_multires.py tests/test_config3.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver$R.log 2>&1 || { tail -20 $O/bench_driver$R.log; exit 1; }
  tail -1 $O/bench_driver$R.log > $O/bench_driver$R.json
  python3 -c "
import json; d=json.load(open('$O/bench_driver$R.json'))
print('driver run $R', round(d['ms_per_step'],4), d['value'], 'pipe', round(d['roofline_pipeline']['frac'],4), 'single', round(d['rank0']['single_stream_pass_ms'],4), 'nofst', round(d['t2d_t1d_only']['ms_per_step'],4), 'fst_cost', round(d['fst_cost'],4), '20+500', round(d['config3_20kb_500kb']['ms_per_step'],4))" | tee -a $O/summary.log
done
