#!/bin/bash
# Config-2 bench with consecutive passes round-robin over 1..4 plans on their own HIP streams
# (bench.py --streams), plus the driver's 20-step command at the chosen setting.
# usage: bash tools/streams_probe.sh <tag> [streams list]
set -o pipefail
TAG=${1:-streams}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in ${2:-1 2 3 4}; do
  timeout -k 10 240 python bench.py --streams $s --no-cpu-baseline --no-hbm-stream > $OUT/bench_s$s.log 2>&1 || { tail -20 $OUT/bench_s$s.log; exit 1; }
  python - "$OUT/bench_s$s.log" "$s" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_ms"]
print(f"streams {sys.argv[2]}: {d['value']:.4g} windows/s  {d['ms_per_step']*1e3:.2f} us/step  "
      f"k_prep {k['k_prep']*1e3:.2f} k_bg_slice {k['k_bg_slice']*1e3:.2f} k_scan_w {k['k_scan_w']*1e3:.2f} us")
EOF
done
