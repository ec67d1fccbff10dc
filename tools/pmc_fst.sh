#!/bin/bash
# VALU / LDS / busy counters of config 3 with the Fst terms on (tools/profile_scan.py ... fst)
set -o pipefail
OUT=gpurun_out/${1:-r01}/pmc_fst
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d $OUT/p1 -o pmc -- python3 tools/profile_scan.py config3 3 fst > $OUT/p1.log 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT/p2 -o pmc -- python3 tools/profile_scan.py config3 3 fst > $OUT/p2.log 2>&1
echo rc=$?
