#!/bin/bash
# per-phase stamps of config 5's kernels (diagnostic build libsfs2d_stamps.so): where k_bg_slice's 25 us go
set -o pipefail
O=gpurun_out/r06al; mkdir -p $O
SFS2D_LIB=$PWD/2dsfs-scan_amd/csrc/libsfs2d_stamps.so timeout -k 10 200 python tools/stamps.py config5b > $O/stamps_config5b.txt 2>&1 && SFS2D_LIB=$PWD/2dsfs-scan_amd/csrc/libsfs2d_stamps.so timeout -k 10 200 python tools/stamps.py config5 >> $O/stamps_config5b.txt 2>&1; rc=$?
cat $O/stamps_config5b.txt; exit $rc
