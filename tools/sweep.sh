#!/bin/bash
# tile / chunk sweep on config 2 (with Fst): k_prep tile size and k_scan_w windows per workgroup
for t in 2048 4096 8192 16384; do
  echo -n "tile=$t "; SFS2D_TILE=$t timeout -k 10 60 python tools/profile_scan.py config2 50 fst || exit 1
done
for c in 8 16 32; do
  echo -n "chunk=$c "; SFS2D_CHUNK=$c timeout -k 10 60 python tools/profile_scan.py config2 50 fst || exit 1
done
