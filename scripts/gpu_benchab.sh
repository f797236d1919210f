#!/bin/bash
# alternating bench A/B of library variants (bench.py values only, no profiler):
# usage: scripts/gpu_benchab.sh <out-tag> <reps> "<bench args>" <variant-tag>...
set -u
OUT=gpurun_out/$1; REPS=$2; ARGS=$3; shift 3
mkdir -p $OUT
REPO=$(pwd)
for rep in $(seq 1 $REPS); do
  for v in main "$@"; do
    if [ $v = main ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_v$v.so; fi
    PHDSLAM_LIB=$LIB timeout -k 10 300 python bench.py --no-cpu-baseline --no-config4-model $ARGS > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail -5 $OUT/b_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${v}_$rep.json'));print('$v rep $rep', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
  done
done
