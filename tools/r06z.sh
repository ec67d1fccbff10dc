#!/bin/bash
# round 6: k_slots_search from interpolated guesses (default) vs plain bisection (SFS2D_SRCH_GUESS=0): the
# slot-path parity tests, then config 4 at full size with the search's slot table, interleaved
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_synth_device.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "slot or generator or supplied or dropin_class or config4 or sims" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
for V in 1 0; do
  echo "== SFS2D_SRCH_GUESS=$V" >> $O/c4.log
  SFS2D_SRCH_GUESS=$V SFS2D_SEG=search timeout -k 10 300 python tools/sims_config4.py 2500 4 2>&1 | grep -v amdgpu.ids | tail -2 >> $O/c4.log || exit 1
done; done
cat $O/c4.log
