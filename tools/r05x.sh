set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_synth_device.py tests/test_fp_sweep.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for R in 1 2; do
  for T in 1 0; do
    echo "== SFS2D_TRI=$T" | tee -a $O/c4.log
    SFS2D_TRI=$T timeout -k 10 300 python tools/sims_config4.py 2500 2 3 2>&1 | grep -v amdgpu.ids | tail -1 | tee -a $O/c4.log || exit 1
  done
done
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log > $O/bench_driver.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/rocprof_bench.log 2>&1 || { tail -20 $O/rocprof_bench.log; exit 1; }
echo done
