#!/bin/bash
# round 6: k_scan_gw's windows per workgroup on config 4 (SFS2D_GWWIN 64 default / 128 / 256 / 32), with its
# LDS ln table filled per workgroup; config 4 at full size, slots by k_slots_search, interleaved
O=gpurun_out/r06aa; mkdir -p $O
for i in 1 2; do
for V in 64 128 256 32; do
  echo "== SFS2D_GWWIN=$V" >> $O/c4.log
  SFS2D_GWWIN=$V SFS2D_SEG=search timeout -k 10 300 python tools/sims_config4.py 2500 4 2>&1 | grep -v amdgpu.ids | tail -2 >> $O/c4.log || exit 1
done; done
cat $O/c4.log
