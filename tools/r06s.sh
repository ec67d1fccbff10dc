#!/bin/bash
# round 6: k_scan_gw with ln(x < 512) in the wave's LDS (default where it costs no occupancy) vs the global ln
# table (SFS2D_LNL=0): the large-grid / sims parity tests, then config 4 at full size, interleaved
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_synth_device.py -x -q --timeout 300 --timeout-method thread -k "large_grid or overcalled or sims or synth or generator or config4 or largest or records_per_chrom or dropin_class" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for V in 1 0; do
  echo "== SFS2D_LNL=$V" >> $O/c4.log
  SFS2D_LNL=$V SFS2D_SEG=search timeout -k 10 300 python tools/sims_config4.py 2500 4 2>&1 | grep -v amdgpu.ids | tail -2 >> $O/c4.log || exit 1
done; done
cat $O/c4.log
