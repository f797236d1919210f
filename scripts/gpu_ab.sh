#!/bin/bash
# alternating A/B of the config-3 bench: libphdslam_base.so (A) vs libphdslam.so (B)
# usage: scripts/gpu_ab.sh <tag> [reps] [extra env for A]
set -u
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
for rep in $(seq 1 ${2:-3}); do
  for v in A B; do
    if [ $v = A ]; then LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_base.so; else LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam.so; fi
    env ${3:-PHD_NONE=1} PHDSLAM_LIB=$LIB timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 200 > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit $?
    python3 -c "import json;d=json.load(open('$OUT/c3_${v}_$rep.json'));print('$v rep $rep:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
  done
done
