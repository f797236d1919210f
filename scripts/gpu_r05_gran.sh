#!/bin/bash
# LDS allocation granularity of the occupancy model: residency timeline (stamps
# builds) and alternating bench A/B at configs 3 and 4 per GPU
set -u
OUT=gpurun_out/r05gran; mkdir -p $OUT
L=$PWD/cuda-phdslam_amd/phdslam
for v in stamps vsg512 vsg1280; do
  f=$L/libphdslam_$v.so
  PHDSLAM_LIB=$f timeout -k 10 200 python scripts/phase_stamps.py --config 3 > $OUT/st3_$v.txt 2>&1 || { tail -5 $OUT/st3_$v.txt; exit 1; }
  echo "$v c3: $(grep 'threads/LDS' $OUT/st3_$v.txt) $(grep 'timeline: launch' $OUT/st3_$v.txt | cut -c1-300)"
done
bash scripts/gpu_benchab.sh r05gran/c3 2 "--steps 300" g512 g1280 || exit 1
bash scripts/gpu_benchab.sh r05gran/c4 2 "--config 4 --particles 4096 --steps 300" g512 g1280 || exit 1
for v in main g512 g1280; do python3 -c "import json;d=json.load(open('$OUT/c3/b_${v}_1.json'));c=d['config'];print('$v c3 lds', c['update_lds_bytes'], 'resident', c['update_resident_workgroups'])"; done
