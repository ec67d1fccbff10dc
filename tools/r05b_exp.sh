set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
for L in "" _m _r _mr; do
  echo "== lib$L" >> $O/exp.log
  SFS2D_LIB=2dsfs-scan_amd/csrc/libsfs2d$L.so timeout -k 10 240 python tools/exp_scan.py config3 - nofst >> $O/exp.log 2>&1 || { echo fail; exit 1; }
done
cat $O/exp.log | grep config3
for F in 1 0; do
  echo "== FUSED=$F" >> $O/streams.log
  SFS2D_FUSED=$F timeout -k 10 240 python tools/exp_streams_cfg3.py 100 fst 1 >> $O/streams.log 2>&1 || exit 1
done
cat $O/streams.log
