#!/bin/bash
# wave-kernel stamps for the stamps build and each ablation build (config 3)
set -u
OUT=gpurun_out/${1:-abl}
mkdir -p $OUT
for x in ${2:-stamps}; do
  if [ "$x" = stamps ]; then LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_stamps.so; else LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_x$x.so; fi
  PHDSLAM_LIB=$LIB timeout -k 10 120 python scripts/wave_stamps.py --config 3 > $OUT/st_$x.log 2>&1 || { tail -n 5 $OUT/st_$x.log; exit 1; }
  echo "=== $x"; grep -v amdgpu.ids $OUT/st_$x.log
done
