#!/bin/bash
# Diagnostics of the config-3 update kernel: phase stamps (stamps build) and
# two PMC passes (VALU / LDS utilisation) on the shipped library.
# usage: scripts/gpu_diag.sh <tag> [stamps] [pmc]
set -u
T=${1:-diag}
REPO=$(pwd)
OUT=$REPO/gpurun_out/$T
mkdir -p $OUT
shift
for what in "$@"; do
  if [ $what = stamps ]; then
    PHDSLAM_LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_stamps.so timeout -k 10 200 python scripts/phase_stamps.py --config 3 > $OUT/stamps_c3.log 2>&1 || { tail -5 $OUT/stamps_c3.log; exit 1; }
    grep -v amdgpu.ids $OUT/stamps_c3.log
  fi
  if [ $what = pmc ]; then
    for ps in a b; do
      if [ $ps = a ]; then C="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES"
      else C="SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM_RD"; fi
      P=$OUT/pmc_$ps
      mkdir -p $P
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P -o run -- python3 $REPO/bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > $P/log.txt 2>&1) || { tail -n 3 $P/log.txt; exit 1; }
      python3 scripts/pmc_summary.py $P | grep -E "update|==" 
    done
  fi
done
exit 0
