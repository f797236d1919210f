#!/bin/bash
# SQ instruction counters of the config-3 update for the product library and ablation builds
set -u
T=${1:-abl}
REPO=$(pwd)
for x in ${2:-prod 12 13 14}; do
  if [ "$x" = prod ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_x$x.so; fi
  OUT=$REPO/gpurun_out/pmc_${T}_$x
  mkdir -p $OUT
  (cd /tmp && export TMPDIR=/tmp && PHDSLAM_WAVE_DEFAULT=1 PHDSLAM_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT -o run -- python3 $REPO/bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/log.txt 2>&1) || { tail -n 3 $OUT/log.txt; exit 1; }
  echo "== $x"; python3 scripts/pmc_summary.py $OUT | grep wave
done
