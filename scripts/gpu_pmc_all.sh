#!/bin/bash
# round-5 PMC reports (HBM traffic, VALU / LDS issue) + kernel stats, every benched shape
set -u
bash scripts/gpu_round_pmc.sh r05pmc_c3 3 || exit 1
bash scripts/gpu_round_pmc.sh r05pmc_c2 2 || exit 1
PARTICLES=4096 bash scripts/gpu_round_pmc.sh r05pmc_c4 4 || exit 1
PARTICLES=8192 bash scripts/gpu_round_pmc.sh r05pmc_c5 5 || exit 1
