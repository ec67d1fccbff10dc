# round-5 measurement session: GPU tests, bench (default and the driver's command), rocprofv3 kernel
# trace of the driver's command, PMC bytes + SQ counters, config 4 (generator slots and segmentation)
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
tail -1 $O/bench_driver.log > $O/bench_driver.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/rocprof_bench.log 2>&1 || { tail -20 $O/rocprof_bench.log; exit 1; }
bash tools/pmc_bench.sh r05s > $O/pmc_bench.log 2>&1 || { tail -20 $O/pmc_bench.log; exit 1; }
bash tools/pmc_k3.sh r05s config3 fst > $O/pmc_k3.log 2>&1 || { tail -20 $O/pmc_k3.log; exit 1; }
timeout -k 10 300 python tools/sims_config4.py 2500 4 3 > $O/sims_config4_generator_slots.txt 2>&1 || { tail -20 $O/sims_config4_generator_slots.txt; exit 1; }
SFS2D_SYNTH_SEG=0 timeout -k 10 300 python tools/sims_config4.py 2500 4 3 > $O/sims_config4_segmentation.txt 2>&1 || { tail -20 $O/sims_config4_segmentation.txt; exit 1; }
echo done
