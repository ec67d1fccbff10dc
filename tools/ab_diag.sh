#!/bin/bash
# A/B diagnostics of the scan kernels: per-config timings, block/wave stamps and SQ counter passes
# for the current library and a comparison build (SFS2D_LIB).
# usage: bash tools/ab_diag.sh <tag> [other.so] [other_stamps.so]
set -o pipefail
TAG=${1:-ab}
OTHER=${2:-2dsfs-scan_amd/csrc/libsfs2d_old.so}
OTHER_ST=${3:-2dsfs-scan_amd/csrc/libsfs2d_old_stamps.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for lib in new old; do
  if [ $lib = new ]; then L=2dsfs-scan_amd/csrc/libsfs2d.so; LS=2dsfs-scan_amd/csrc/libsfs2d_stamps.so; else L=$OTHER; LS=$OTHER_ST; fi
  for c in config2 config3; do
    SFS2D_LIB=$L timeout -k 10 180 python tools/profile_scan.py $c 20 fst >> $OUT/profile_$lib.log 2>&1 || { cat $OUT/profile_$lib.log; exit 1; }
    SFS2D_LIB=$LS timeout -k 10 180 python tools/stamps.py $c >> $OUT/stamps_$lib.log 2>&1 || { cat $OUT/stamps_$lib.log; exit 1; }
  done
  P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU"
  P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
  P3="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAVES"
  for p in 1 2 3; do
    eval C=\$P$p
    SFS2D_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/pmc_$lib/p$p -o pmc -- python3 tools/profile_scan.py config3 3 fst > $OUT/pmc_${lib}_p$p.log 2>&1 || { tail -5 $OUT/pmc_${lib}_p$p.log; echo "pmc pass $p failed (continuing)"; }
  done
  python3 tools/pmc_summary.py $OUT/pmc_$lib > $OUT/pmc_config3_$lib.csv 2>&1 || true
done
cat $OUT/profile_new.log $OUT/profile_old.log | grep -v amdgpu.ids
grep -v "^ *[0-9]" $OUT/stamps_new.log | grep -v amdgpu.ids
grep -v "^ *[0-9]" $OUT/stamps_old.log | grep -v amdgpu.ids
cat $OUT/pmc_config3_new.csv $OUT/pmc_config3_old.csv
