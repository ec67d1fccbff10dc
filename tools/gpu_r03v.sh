#!/bin/bash
# k_scan_gw with pipelined row pairs (lp loads issued one pair ahead; build/ab/lib_GWP.so): GPU parity of
# the large-grid paths, config 4 / config 5 timings against the tree's build; k_scan_w phase stamps
set -o pipefail
OUT=gpurun_out/r03v
mkdir -p $OUT
export TMPDIR=/tmp
SFS2D_LIB=build/ab/lib_GWP.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "parity or sims or multires or synth" > $OUT/tests_gwp.log 2>&1 || { tail -30 $OUT/tests_gwp.log; exit 1; }
tail -1 $OUT/tests_gwp.log
for r in 1 2; do
  for L in 2dsfs-scan_amd/csrc/libsfs2d.so build/ab/lib_GWP.so; do
    echo "== $L" >> $OUT/cfg4.log
    SFS2D_LIB=$L timeout -k 10 300 python tools/sims_config4.py 2500 1 3 2>&1 | grep -v amdgpu.ids >> $OUT/cfg4.log || exit 1
    echo -n "$(basename $L) config5: " >> $OUT/cfg5.log
    SFS2D_LIB=$L timeout -k 10 120 python tools/profile_scan.py config5 30 2>&1 | grep nrec >> $OUT/cfg5.log || exit 1
  done
done
cat $OUT/cfg4.log $OUT/cfg5.log
for C in config2 config3; do
  SFS2D_LIB=build/ab/lib_STAMPS.so timeout -k 10 120 python tools/stamps.py $C 2>&1 | grep -v amdgpu.ids >> $OUT/stamps.log || exit 1
done
cat $OUT/stamps.log
