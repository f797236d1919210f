#!/bin/bash
# A/B of the per-step overhead at config 3: single-launch normalise+resample
# (PHD_RS_SINGLE_MAX) and the predict fused into part A (PHD_FUSE_PREDICT)
set -u
mkdir -p gpurun_out/ovh
for v in "0 2048" "0 4096" "1 2048" "1 4096"; do
  set -- $v
  PHD_FUSE_PREDICT=$1 PHD_RS_SINGLE_MAX=$2 timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/ovh/b_$1_$2.json 2> gpurun_out/ovh/b_$1_$2.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/ovh/b_$1_$2.json'));print('fuse $1 single_max $2:', d['value'], 'steps/s; ms/step', d['ms_per_step'], 'update ms', d['roofline']['avg_kernel_ms'])"
done
