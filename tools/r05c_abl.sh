set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
for L in "" _xf _abl1 _abl2 _abl4 _abl8 _abl16 _abl32 _abl63 _xf ""; do
  SFS2D_LIB=2dsfs-scan_amd/csrc/libsfs2d$L.so timeout -k 10 120 python tools/ktime.py fst 7 2>&1 | grep -v amdgpu.ids | tee -a $O/abl.log || exit 1
done
for L in "" _abl1; do
  SFS2D_LIB=2dsfs-scan_amd/csrc/libsfs2d$L.so timeout -k 10 120 python tools/ktime.py fst 7 config2 2>&1 | grep -v amdgpu.ids | tee -a $O/abl.log || exit 1
done
