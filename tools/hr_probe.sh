#!/bin/bash
# k_prep LDS histogram copies per word: 4 (now 1 by default) vs 4 (SFS2D_HR=4)
mkdir -p gpurun_out/hr
for hr in "" 4; do
  for c in config2 config3; do
    echo "hr=${hr:-default} $c" >> gpurun_out/hr/log.txt
    SFS2D_HR=$hr timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> gpurun_out/hr/log.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/hr/log.txt
