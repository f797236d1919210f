#!/bin/bash
# PMC passes + kernel stats of configs 4 / 5 per GPU and 2 (closing evidence after the occupancy fix)
set -u
T=${1:-r05fin5}
PARTICLES=4096 bash scripts/gpu_round_pmc.sh ${T}_pmc_c4 4 || exit 1
PARTICLES=8192 bash scripts/gpu_round_pmc.sh ${T}_pmc_c5 5 || exit 1
bash scripts/gpu_round_pmc.sh ${T}_pmc_c2 2 || exit 1
