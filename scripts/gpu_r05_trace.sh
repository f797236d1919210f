#!/bin/bash
# kernel trace (start / end of every launch) of the config-3 bench, per library variant
set -u
OUT=gpurun_out/r05trace; mkdir -p $OUT
REPO=$(pwd)
for v in "$@"; do
  if [ $v = main ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_v$v.so; fi
  (cd /tmp && export TMPDIR=/tmp && PHDSLAM_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $REPO/$OUT/tr_$v -o run -- python3 $REPO/bench.py --no-cpu-baseline --no-config4-model --steps 60 --warmup 10 > $REPO/$OUT/b_$v.json 2> $REPO/$OUT/b_$v.err) || { tail -5 $OUT/b_$v.err; exit 1; }
  f=$(find $OUT/tr_$v -name '*kernel_trace.csv' | head -1); cp $f $OUT/trace_$v.csv
done
