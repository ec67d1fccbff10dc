#!/bin/bash
# time one config across library variants: bash tools/variants.sh <config> <iters> [fst] -- lib1.so lib2.so ...
set -o pipefail
C=$1; I=$2; F=$3; shift 4
for lib in "$@"; do
  echo -n "$(basename $lib) "; SFS2D_LIB=$lib timeout -k 10 90 python tools/profile_scan.py $C $I $F || exit 1
done
