#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of the config-3 update
# for the shipped library and each timing-ablation build (build.py --ablation N),
# plus the shipped library's L2 hit / miss counts: the per-phase byte
# attribution of part C.  Parse with scripts/traffic_ablate.py <tag>.
# usage: scripts/gpu_traffic_ablate.sh <tag> <lib> [<lib> ...]   (lib: file under cuda-phdslam_amd/phdslam)
set -u
TAG=${1:-tab}; shift
REPO=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  for P in FETCH_SIZE WRITE_SIZE; do
    OUT=$REPO/gpurun_out/$TAG/$v/$P
    mkdir -p "$OUT"
    PHDSLAM_LIB=$REPO/cuda-phdslam_amd/phdslam/$v timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d "$OUT" -o run -- python3 "$REPO/bench.py" --config 3 --steps 20 --warmup 2 --no-cpu-baseline --no-config4-model > "$OUT/log.txt" 2>&1 || { tail -3 "$OUT/log.txt"; exit 1; }
    echo "done $v $P"
  done
done
OUT=$REPO/gpurun_out/$TAG/l2
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT" -o run -- python3 "$REPO/bench.py" --config 3 --steps 20 --warmup 2 --no-cpu-baseline --no-config4-model > "$OUT/log.txt" 2>&1 || { tail -3 "$OUT/log.txt"; exit 1; }
echo done l2
