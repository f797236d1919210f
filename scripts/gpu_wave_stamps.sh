#!/bin/bash
# wave kernel phase stamps (diagnostic build) for the given configs
set -u
OUT=gpurun_out/${1:-wst}
mkdir -p $OUT
for c in ${2:-3}; do
  timeout -k 10 200 python scripts/wave_stamps.py --config $c ${3:-} > $OUT/st$c.log 2>&1 || { tail -5 $OUT/st$c.log; exit 1; }
  cat $OUT/st$c.log
done
if [ -n "${4:-}" ]; then
  for x in $4; do
    PHDSLAM_LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_x$x.so timeout -k 10 200 python scripts/wave_stamps.py --config 3 > $OUT/st3_x$x.log 2>&1 || { tail -5 $OUT/st3_x$x.log; exit 1; }
    echo "== experiment $x"; cat $OUT/st3_x$x.log
  done
fi
