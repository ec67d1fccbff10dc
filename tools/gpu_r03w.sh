#!/bin/bash
# build/ab/lib_SB8.so = lib_OFF + the 2D atomic exec-masked (no trash words) and 8-window batches;
# build/ab/lib_OFF.so = c94585e: k_scan_w prologue loads in flight together, k_scan_gw pipelined
# pairs and three-sum reduce-scatter, row offsets as one base + immediates (no VGPR spills): full GPU
# suite on it, then A/B against the in-tree build (eb150c8) on configs 2 / 3 / 4 / 5
set -o pipefail
OUT=gpurun_out/r03w
mkdir -p $OUT
export TMPDIR=/tmp
SFS2D_LIB=build/ab/lib_SB8.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/tests_sb8.log 2>&1 || { tail -30 $OUT/tests_sb8.log; exit 1; }
tail -1 $OUT/tests_sb8.log
for r in 1 2; do
  for L in 2dsfs-scan_amd/csrc/libsfs2d.so build/ab/lib_OFF.so build/ab/lib_SB8.so; do
    for C in "config2 30 fst" "config2 30" "config3 30 fst" "config3 30" "config5 30"; do
      echo -n "$(basename $L) $C: " >> $OUT/ab.log
      SFS2D_LIB=$L timeout -k 10 120 python tools/profile_scan.py $C 2>&1 | grep nrec >> $OUT/ab.log || exit 1
    done
  done
done
cat $OUT/ab.log
for r in 1; do
  for L in 2dsfs-scan_amd/csrc/libsfs2d.so build/ab/lib_OFF.so build/ab/lib_SB8.so; do
    echo "== $L" >> $OUT/cfg4.log
    SFS2D_LIB=$L timeout -k 10 300 python tools/sims_config4.py 2500 1 3 2>&1 | grep -v amdgpu.ids >> $OUT/cfg4.log || exit 1
  done
done
cat $OUT/cfg4.log
for L in build/ab/lib_OFF.so build/ab/lib_SB8.so; do
  echo "== $L" >> $OUT/streams.log
  for F in "fst 1" "fst 0" "nofst 1"; do echo "-- $F" >> $OUT/streams.log; SFS2D_LIB=$L timeout -k 10 200 python tools/exp_streams_cfg3.py 24 $F >> $OUT/streams.log 2>&1 || exit 1; done
done
grep -v amdgpu.ids $OUT/streams.log
