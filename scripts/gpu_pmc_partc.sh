#!/bin/bash
# stall / issue breakdown of the config-3 update kernels (two SQ passes + clock)
# usage: scripts/gpu_pmc_partc.sh <tag> [lib]
set -u
TAG=${1:-pmcc}; LIBN=${2:-libphdslam.so}
REPO=$(pwd)
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SMEM"
P3="GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  OUT=$REPO/gpurun_out/$TAG/p$i
  mkdir -p "$OUT"
  (cd /tmp && export TMPDIR=/tmp && PHDSLAM_LIB=$REPO/cuda-phdslam_amd/phdslam/$LIBN timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT" -o run -- python3 "$REPO/bench.py" --config 3 --steps 20 --warmup 2 --no-cpu-baseline --no-config4-model > "$OUT/log.txt" 2>&1) || { tail -5 $OUT/log.txt; exit 1; }
  python3 scripts/pmc_summary.py "$OUT" | grep -i "update_cphd\|cphd_terms"
done
