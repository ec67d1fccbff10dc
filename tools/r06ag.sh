#!/bin/bash
# one config-3 scan cut into chromosome groups alternating over 2 streams vs the whole genome as one plan
set -o pipefail
O=gpurun_out/r06ag; mkdir -p $O
timeout -k 10 300 python -u tools/exp_chunked_pass.py 30 0,1 > $O/chunked.txt 2>&1; rc=$?; cat $O/chunked.txt; exit $rc
