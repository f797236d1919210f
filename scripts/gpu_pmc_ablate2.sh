#!/bin/bash
# LDS / VALU counters of the config-3 wave update for ablation builds
set -u
T=${1:-abl}
REPO=$(pwd)
for x in ${2:-16 17}; do
  LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_x$x.so
  for ps in a b; do
    if [ $ps = a ]; then C="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
    else C="SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_INSTS_VMEM_RD"; fi
    OUT=$REPO/gpurun_out/pmc_${T}_${x}_$ps
    mkdir -p $OUT
    (cd /tmp && export TMPDIR=/tmp && PHDSLAM_WAVE_DEFAULT=1 PHDSLAM_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT -o run -- python3 $REPO/bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/log.txt 2>&1) || { tail -n 3 $OUT/log.txt; exit 1; }
    echo "== $x $ps"; python3 scripts/pmc_summary.py $OUT | grep wave
  done
done
