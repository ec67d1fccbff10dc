#!/bin/bash
# buffer-load rows (per-window descriptors): parity subset + config 2/3 timings, then config 4 (sims, k_scan_gw)
set -o pipefail
bash tools/gpu_quick_ab.sh r03p "parity or fst or multires or config or sims or gw" || exit 1
timeout -k 10 300 python tools/sims_config4.py 2500 2 3 > gpurun_out/r03p/sims_config4.txt 2>&1 || { tail -5 gpurun_out/r03p/sims_config4.txt; exit 1; }
tail -3 gpurun_out/r03p/sims_config4.txt
