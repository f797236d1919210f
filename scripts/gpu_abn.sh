#!/bin/bash
# alternating N-way comparison of the config-3 bench over library variants
# usage: scripts/gpu_abn.sh <tag> <reps> <lib> [<lib> ...]   (lib: path relative to cuda-phdslam_amd/phdslam)
set -u
OUT=gpurun_out/${1:-abn}
REPS=${2:-3}
shift 2
mkdir -p $OUT
for rep in $(seq 1 $REPS); do
  for v in "$@"; do
    LIB=$PWD/cuda-phdslam_amd/phdslam/$v
    PHDSLAM_LIB=$LIB timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 200 > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit $?
    python3 -c "import json;d=json.load(open('$OUT/c3_${v}_$rep.json'));print('$v rep $rep:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
  done
done
