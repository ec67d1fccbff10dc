#!/bin/bash
# after the k_scan_w VALU trims: A/B without Fst and config 2 (HEAD's build vs the tree's), SQ / byte
# counters of config 3 with Fst, overlapped config-3 passes, config 4 (k_scan_gw trims)
set -o pipefail
OUT=gpurun_out/r03t
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for L in build/ab/lib_HEAD.so 2dsfs-scan_amd/csrc/libsfs2d.so build/ab/lib_LPF.so; do
    for C in "config3 30" "config3 30 fst" "config2 30"; do
      echo -n "$(basename $L) $C: " >> $OUT/ab.log
      SFS2D_LIB=$L timeout -k 10 120 python tools/profile_scan.py $C 2>&1 | grep nrec >> $OUT/ab.log || exit 1
    done
  done
done
cat $OUT/ab.log
for L in build/ab/lib_HEAD.so 2dsfs-scan_amd/csrc/libsfs2d.so; do
  echo "== $L" >> $OUT/streams.log
  for F in fst nofst; do echo "-- $F, cap 1" >> $OUT/streams.log; SFS2D_LIB=$L timeout -k 10 200 python tools/exp_streams_cfg3.py 24 $F 1 >> $OUT/streams.log 2>&1 || exit 1; done
done
cat $OUT/streams.log
bash tools/pmc_k3.sh r03t config3 fst || exit 1
timeout -k 10 300 python tools/sims_config4.py 2500 2 3 > $OUT/sims_config4.txt 2>&1 || { tail -5 $OUT/sims_config4.txt; exit 1; }
tail -3 $OUT/sims_config4.txt
