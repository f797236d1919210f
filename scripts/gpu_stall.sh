#!/bin/bash
# stall breakdown of the config-3 update kernels: wait/active cycles, VALU lane use, LDS conflicts
PASSES_A="valu:SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VALU"
PASSES_B="lds:SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS"
PASSES="$PASSES_A" bash scripts/gpu_icache.sh ${1:-stall}_a && PASSES="$PASSES_B" bash scripts/gpu_icache.sh ${1:-stall}_b
