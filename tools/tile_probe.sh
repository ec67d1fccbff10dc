#!/bin/bash
# k_prep tile size (SFS2D_TILE) after the one-copy LDS histogram: config 2 and config 3
mkdir -p gpurun_out/tile
for t in 2048 3072 4096 8192; do
  echo "tile=$t config2" >> gpurun_out/tile/log.txt
  SFS2D_TILE=$t timeout -k 10 180 python tools/profile_scan.py config2 20 fst >> gpurun_out/tile/log.txt 2>&1 || exit 1
done
for t in 16384 32768; do
  echo "tile=$t config3" >> gpurun_out/tile/log.txt
  SFS2D_TILE=$t timeout -k 10 180 python tools/profile_scan.py config3 20 fst >> gpurun_out/tile/log.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/tile/log.txt
