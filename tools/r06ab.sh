#!/bin/bash
# round 6: one rank's config-3 share at N = 4 / 8 (8 / 4 chromosomes: k_prep tiles of 8k SNPs, below the joint
# histogram's 16k gate) with the joint histogram forced on (SFS2D_JNT=1) vs the default (three atomics), and
# N = 2 (16 chromosomes: 16k tiles, joint by default) vs SFS2D_JNT=0; tools/exp_streams_cfg3.py, interleaved
O=gpurun_out/r06ab; mkdir -p $O
for i in 1 2; do
for C in 8 4 16; do
for J in d 1 0; do
  if [ $J = d ]; then unset SFS2D_JNT; else export SFS2D_JNT=$J; fi
  echo "== chromosomes $C SFS2D_JNT=$J" >> $O/share.txt
  timeout -k 10 200 python tools/exp_streams_cfg3.py 40 fst 1 $C 2>> $O/share.err | grep "streams 2" >> $O/share.txt || { tail -20 $O/share.err; exit 1; }
done; done; done
unset SFS2D_JNT
cat $O/share.txt
