#!/bin/bash
# SQ counter passes over the large-grid scan (config 4 shape, 250 replicates generated on the device)
# and over config 3 (k_scan_w), one counter group per run, kernel trace only.
# usage: bash tools/pmc_gw.sh <tag> [4]   (4: the config-4 passes only)
set -o pipefail
TAG=${1:-gw}
export TMPDIR=/tmp
run() {  # outdir name cmd-args... -- counters via PMC env
  local out=$1 name=$2; shift 2
  mkdir -p $out
  timeout -k 10 240 rocprofv3 --pmc $PMC --output-format csv -d $out/$name -o pmc -- "$@" > $out/$name.log 2>&1
}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU"
P2="SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
O4=gpurun_out/$TAG/pmc_config4
O3=gpurun_out/$TAG/pmc_config3
PMC=$P1 run $O4 p1 python3 tools/sims_config4.py 250 1 3 &&
PMC=$P2 run $O4 p2 python3 tools/sims_config4.py 250 1 3 &&
PMC=FETCH_SIZE run $O4 p3 python3 tools/sims_config4.py 250 1 3 &&
python3 tools/pmc_summary.py $O4 > gpurun_out/$TAG/pmc_config4.csv &&
if [ "$2" = 4 ]; then echo "rc=0"; exit 0; fi &&
PMC=$P1 run $O3 p1 python3 tools/profile_scan.py config3 3 fst &&
PMC=$P2 run $O3 p2 python3 tools/profile_scan.py config3 3 fst &&
python3 tools/pmc_summary.py $O3 > gpurun_out/$TAG/pmc_config3.csv
echo "rc=$?"
