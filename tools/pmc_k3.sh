#!/bin/bash
# PMC passes (one counter group per run; no trace domains besides the kernel trace) over one config.
# usage: bash tools/pmc_k3.sh <tag> <config>
set -o pipefail
TAG=${1:-r01}; CFG=${2:-config3}; FST=${3:-}
OUT=gpurun_out/$TAG/pmc_$CFG$FST
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 tools/profile_scan.py $CFG 3 $FST > $OUT/$name.log 2>&1
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU &&
run p2 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_SMEM &&
run p3 FETCH_SIZE &&
run p4 WRITE_SIZE &&
run p5 GRBM_GUI_ACTIVE GRBM_COUNT
echo "rc=$?"
