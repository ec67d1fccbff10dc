set -o pipefail
mkdir -p gpurun_out/occ
for pad in 0 4096 10240 18432 32768; do
  echo "pad $pad" >> gpurun_out/occ/log.txt
  SFS2D_GW_PAD=$pad timeout -k 10 200 python -u tools/sims_config4.py 1000 1 5 >> gpurun_out/occ/log.txt 2>&1 || exit 1
done
cat gpurun_out/occ/log.txt
