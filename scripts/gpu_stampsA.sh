#!/bin/bash
# CPHD part A phase stamps at config 3
set -u
OUT=gpurun_out/${1:-stampsA}
mkdir -p $OUT
timeout -k 10 300 python scripts/phase_stamps.py --config 3 --part A > $OUT/stampsA_c3.txt 2>&1
rc=$?; head -20 $OUT/stampsA_c3.txt; exit $rc
