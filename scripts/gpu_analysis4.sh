#!/bin/bash
# Round-4 close: the bound analysis inputs on the final kernels — stall / VALU
# lane / LDS counters of the config-3 update (gpu_stall.sh), part C and part A
# phase stamps (PHD_STAMPS builds).
# usage: scripts/gpu_analysis4.sh <tag>
set -u
T=${1:-r04fin_an}
OUT=gpurun_out/$T
mkdir -p $OUT
bash scripts/gpu_stall.sh $T || exit $?
timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/stampsC_c3.txt 2>&1 || { tail -5 $OUT/stampsC_c3.txt; exit 1; }
cat $OUT/stampsC_c3.txt
timeout -k 10 300 python scripts/phase_stamps.py --config 3 --part A > $OUT/stampsA_c3.txt 2>&1 || { tail -5 $OUT/stampsA_c3.txt; exit 1; }
cat $OUT/stampsA_c3.txt
