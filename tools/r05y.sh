set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/sims_config4.py 2500 4 3 > $O/sims_config4_generator_slots.txt 2>&1 || { tail -20 $O/sims_config4_generator_slots.txt; exit 1; }
SFS2D_SYNTH_SEG=0 timeout -k 10 300 python tools/sims_config4.py 2500 4 3 > $O/sims_config4_segmentation.txt 2>&1 || { tail -20 $O/sims_config4_segmentation.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c4 -- python3 tools/sims_config4.py 2500 2 2 > $O/rocprof_c4.log 2>&1 || { tail -20 $O/rocprof_c4.log; exit 1; }
echo done
