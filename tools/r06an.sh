#!/bin/bash
# k_bg_slice with the 1D-spectrum block dispatched first (libsfs2d.so) vs as each row's last block
# (libsfs2d_base.so, the previous build): background parity tests, then config 5 / config 2 in the bench, interleaved
set -o pipefail
O=gpurun_out/r06an; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do for v in new base; do
  L=$PWD/2dsfs-scan_amd/csrc/libsfs2d.so; [ $v = base ] && L=$PWD/2dsfs-scan_amd/csrc/libsfs2d_base.so
  SFS2D_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-variants --no-e2e --no-cpu-baseline > $O/bench_${v}_$i.log 2>&1 || { tail -20 $O/bench_${v}_$i.log; exit 1; }
  tail -1 $O/bench_${v}_$i.log > $O/bench_${v}_$i.json
  python -c "import json;d=json.load(open('$O/bench_${v}_$i.json'));c=d['config5_snp_windows'];c2=d['config2_weak'];print('$v', 'c5', round(c['ms_per_step'],5), c['single_stream_pass_ms'], '| c2 %.3e'%c2['value'], c2['single_stream_pass_ms'], '| c3', round(d['ms_per_step'],4))"
done; done
