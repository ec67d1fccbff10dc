#!/bin/bash
# tile / chunk sweep on config 2 (with Fst): k_prep tile size and k_scan_w workgroups
for t in 1024 2048 4096 8192; do
  echo -n "tile=$t "; SFS2D_TILE=$t timeout -k 10 60 python tools/profile_scan.py config2 100 fst || exit 1
done
for c in 128 256 384 512; do
  echo -n "wgs=$c "; SFS2D_WGS=$c timeout -k 10 60 python tools/profile_scan.py config2 100 fst || exit 1
done
