#!/bin/bash
# PMC passes (one rocprofv3 run per pass) over the config-3 bench, wave kernel.
set -u
T=${1:-pmcw}
timeout -s KILL 120 bash scripts/pmc_update.sh 3 ${T}_a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
timeout -s KILL 120 bash scripts/pmc_update.sh 3 ${T}_b SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH || exit 1
timeout -s KILL 120 bash scripts/pmc_update.sh 3 ${T}_c SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INST_LEVEL_LDS || echo "pass c failed"
python3 scripts/pmc_summary.py gpurun_out/pmc_c3_${T}_a gpurun_out/pmc_c3_${T}_b gpurun_out/pmc_c3_${T}_c 2>&1 | grep -E "==|wave"
cat gpurun_out/pmc_c3_${T}_c/log.txt | tail -5
