#!/bin/bash
# part C A/B at config 3 (births): cell walk over four records per thread
# (K <= 1024) and 64x32 lattice variants; stamps of the shipped vs four-record
set -u
OUT=gpurun_out/r05hpa
mkdir -p $OUT
bash scripts/gpu_variants.sh r05hp 3 hp > $OUT/variants.txt 2>&1 || { cat $OUT/variants.txt; exit 1; }
cat $OUT/variants.txt
