set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 100 --timeout-method thread -k "config3 or scan_kernels_agree or fst_low" > $O/quick.log 2>&1; tail -3 $O/quick.log
for E in 1 0 1 0; do
  SFS2D_ONEPASS=$E timeout -k 10 120 python tools/ktime.py fst 7 2>&1 | grep -v amdgpu.ids | sed "s/^/onepass=$E /" | tee -a $O/kt.log || exit 1
done
for E in 1 0; do
  echo "== ONEPASS=$E" >> $O/streams.log
  SFS2D_ONEPASS=$E timeout -k 10 240 python tools/exp_streams_cfg3.py 100 fst 1 >> $O/streams.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/streams.log
bash tools/gpu.sh r05e tests
