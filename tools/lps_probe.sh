#!/bin/bash
# k_bg_slice: pairwise leaves per slice (SFS2D_LPS = 4 default, 2, 1) on configs 2 and 3
mkdir -p gpurun_out/lps
for l in 4 2 1; do
  for c in config2 config3; do
    echo "lps=$l $c" >> gpurun_out/lps/log.txt
    SFS2D_LPS=$l timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> gpurun_out/lps/log.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids gpurun_out/lps/log.txt
