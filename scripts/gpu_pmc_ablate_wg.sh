#!/bin/bash
# VALU / SALU / LDS instruction counts of the config-3 workgroup update for the
# shipped library and ablation builds (libphdslam_k<X>.so): instructions per phase
set -u
T=${1:-pabl}
REPO=$(pwd)
OUT=$REPO/gpurun_out/$T
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1) || true
grep -o "SQ_INSTS_VALU[A-Z0-9_]*\|SQ_INSTS_[A-Z0-9_]*" $OUT/counters.txt | sort -u | tr '\n' ' '; echo
for x in base ${2:-2 3 4}; do
  if [ $x = base ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_k$x.so; fi
  C=${3:-"SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES"}
  P=$OUT/pmc_$x
  mkdir -p $P
  (cd /tmp && export TMPDIR=/tmp && PHDSLAM_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $P -o run -- python3 $REPO/bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline > $P/log.txt 2>&1) || { tail -n 3 $P/log.txt; exit 1; }
  echo "== $x"; python3 scripts/pmc_summary.py $P | grep update
done
exit 0
