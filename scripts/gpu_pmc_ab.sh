#!/bin/bash
# instruction-count PMC pass of the config-3 update for each library variant
# usage: scripts/gpu_pmc_ab.sh <tag> <lib> [<lib> ...]   (lib: file name under cuda-phdslam_amd/phdslam)
set -u
TAG=${1:-pmcab}; shift
REPO=$(pwd)
for v in "$@"; do
  OUT=$REPO/gpurun_out/$TAG/$v
  mkdir -p "$OUT"
  (cd /tmp && export TMPDIR=/tmp && PHDSLAM_LIB=$REPO/cuda-phdslam_amd/phdslam/$v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d "$OUT" -o run -- python3 "$REPO/bench.py" --config 3 --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/log.txt" 2>&1) || exit $?
  echo "== $v"; python3 scripts/pmc_summary.py "$OUT" | grep -i "update_cphd_c\|update_cphd_a"
done
