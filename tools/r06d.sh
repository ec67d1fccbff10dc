#!/bin/bash
# round 6: k_slots_search (config 4's slot table by binary search) -- parity tests, then config 4 with the
# three slot-table paths (generator offsets / search / k_prep)
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_synth_device.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
for S in search prep auto; do
  echo "== SFS2D_SEG=$S" >> $O/c4.log
  SFS2D_SEG=$S timeout -k 10 300 python tools/sims_config4.py 2500 4 3 >> $O/c4.log 2>&1 || { tail -20 $O/c4.log; exit 1; }
done
tail -5 $O/pytest.log; grep -E "==|config 4" $O/c4.log
