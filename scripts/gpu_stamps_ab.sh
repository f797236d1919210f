#!/bin/bash
# part C phase stamps at config 3 for each stamps-library variant
# usage: scripts/gpu_stamps_ab.sh <tag> <lib> [<lib> ...]   (lib: file name under cuda-phdslam_amd/phdslam)
set -u
OUT=gpurun_out/${1:-stab}; shift
mkdir -p $OUT
for v in "$@"; do
  PHDSLAM_LIB=$PWD/cuda-phdslam_amd/phdslam/$v timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/$v.txt 2>&1 || exit $?
done
