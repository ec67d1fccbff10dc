set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
for rep in 1 2; do
for L in "" _m _r _mr; do
  SFS2D_LIB=2dsfs-scan_amd/csrc/libsfs2d$L.so timeout -k 10 120 python tools/ktime.py fst 7 2>&1 | grep -v amdgpu.ids | tee -a $O/ab.log || exit 1
done
done
bash tools/gpu.sh r05d tests
