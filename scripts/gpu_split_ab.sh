#!/bin/bash
# A/B of the update split over streams (PHD_UPD_SPLIT) at configs 3 and 2
set -u
mkdir -p gpurun_out/split
for c in 3 2; do
  for k in 1 2 3 4; do
    PHD_UPD_SPLIT=$k timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/split/b${c}_${k}.json 2> gpurun_out/split/b${c}_${k}.err || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/split/b${c}_${k}.json'));print('config $c split $k:', d['value'], 'steps/s; ms/step', d['ms_per_step'], 'update ms', d['roofline']['avg_kernel_ms'])"
  done
done
