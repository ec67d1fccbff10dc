#!/bin/bash
# round 6: k_prep's cost of the position bytes (ablation builds, synthetic window ids: 1024 reads 2 B of
# position per SNP, 2048 none, 64 no LDS histogram atomics, 1088 both 1024 and 64), config 3 with Fst
O=gpurun_out/r06h; mkdir -p $O
V=2dsfs-scan_amd/csrc/variants
export SFS2D_ALLOW_ABLATION=1
for i in 1 2; do
for L in 2dsfs-scan_amd/csrc/libsfs2d.so $V/libsfs2d_abl1024.so $V/libsfs2d_abl2048.so $V/libsfs2d_abl64.so $V/libsfs2d_abl1088.so; do
  SFS2D_LIB=$L timeout -k 10 120 python tools/ktime.py fst 7 >> $O/ktime.txt 2>> $O/ktime.err || { tail -20 $O/ktime.err; exit 1; }
done; done
cat $O/ktime.txt
