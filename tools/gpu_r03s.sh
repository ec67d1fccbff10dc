#!/bin/bash
# round 3, session 2: full GPU suite on the working tree, A/B of k_scan_w's Fst (alt, ref) table against
# HEAD's build (build/ab/lib_HEAD.so), then the bench and a rocprofv3 kernel trace of it
set -o pipefail
OUT=gpurun_out/r03s
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for r in 1 2; do
  for L in build/ab/lib_HEAD.so build/ab/lib_FT.so build/ab/lib_W5.so build/ab/lib_G1.so 2dsfs-scan_amd/csrc/libsfs2d.so; do
    for C in "config3 30 fst" "config2 30 fst"; do
      echo -n "$(basename $L) $C: " >> $OUT/ab.log
      SFS2D_LIB=$L timeout -k 10 120 python tools/profile_scan.py $C 2>&1 | grep nrec >> $OUT/ab.log || exit 1
    done
  done
done
cat $OUT/ab.log
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 bench.py --no-cpu-baseline --no-e2e > $OUT/rocprof_bench.log 2>&1 || { tail -20 $OUT/rocprof_bench.log; exit 1; }
find $OUT/prof -name "*stats*"
