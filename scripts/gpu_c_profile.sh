#!/bin/bash
# part C of the config-3 CPHD update: phase stamps, ablation timings and VALU counts
set -u
T=${1:-cprof}
bash scripts/gpu_diag.sh $T stamps || exit 1
bash scripts/gpu_ablate_wg.sh ${T}_abl "${2:-3 4 7 8 9}" || exit 1
bash scripts/gpu_pmc_ablate_wg.sh ${T}_pmc "${2:-3 4 7 8 9}" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" || exit 1
