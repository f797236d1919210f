#!/bin/bash
# A/B (alternating) of the CV predict fused into part A at config 3 (PHD_FUSE_PREDICT)
set -u
mkdir -p gpurun_out/fab
i=0
for f in 0 1 0 1 0 1; do
  i=$((i+1))
  PHD_FUSE_PREDICT=$f timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 400 --warmup 40 > gpurun_out/fab/b_${f}_$i.json 2> gpurun_out/fab/b_${f}_$i.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/fab/b_${f}_$i.json'));print('fuse $f:', d['value'], 'steps/s; ms/step', d['ms_per_step'], 'update ms', d['roofline']['avg_kernel_ms'])"
done
