#!/bin/bash
# part C A/B at config 3 (births): cell walk over four records per thread
# (K <= 1024) and 64x32 lattice variants; stamps of the shipped vs four-record
set -u
OUT=gpurun_out/r05em
mkdir -p $OUT
bash scripts/gpu_variants.sh r05em 3 em > $OUT/variants.txt 2>&1 || { cat $OUT/variants.txt; exit 1; }
cat $OUT/variants.txt
bash scripts/gpu_stamps_ab.sh r05em libphdslam_vsem.so || exit 1
grep -h "merge\|total\|cand:\|per-WG" $OUT/libphdslam_vsem.so.txt | head -60
