#!/bin/bash
# k_fst_win (attached sliced Fst plans) with the current library vs another build: rocprofv3 kernel
# stats of tools/multires_time.py config2 (20 kb base + 500 kb attached, both with Fst).
# usage: bash tools/fst_win_cmp.sh <outdir> <other.so>
set -o pipefail
OUT=$1; OTHER=$2
mkdir -p $OUT
export TMPDIR=/tmp
for v in new old; do
  if [ $v = new ]; then L=2dsfs-scan_amd/csrc/libsfs2d.so; else L=$OTHER; fi
  SFS2D_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o fw -- python3 tools/multires_time.py config2 50 > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  f=$(find $OUT/$v -name "fw_kernel_stats.csv" | head -1)
  echo "== $v"; grep -E "Name|k_fst_win|k_fst_agg|k_slots_bp" $f | cut -c1-200
done
