#!/bin/bash
# the stamps and PMC passes of the round-5 closing evidence
set -u
T=${1:-r05fin}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/stamps_c3_partC.txt 2>&1 || { tail -5 $OUT/stamps_c3_partC.txt; exit 1; }
timeout -k 10 300 python scripts/phase_stamps.py --config 3 --part A > $OUT/stamps_c3_partA.txt 2>&1 || { tail -5 $OUT/stamps_c3_partA.txt; exit 1; }
bash scripts/gpu_round_pmc.sh ${T}_pmc_c3 3 || exit 1
PARTICLES=4096 bash scripts/gpu_round_pmc.sh ${T}_pmc_c4 4 || exit 1
PARTICLES=8192 bash scripts/gpu_round_pmc.sh ${T}_pmc_c5 5 || exit 1
bash scripts/gpu_round_pmc.sh ${T}_pmc_c2 2 || exit 1
