#!/bin/bash
# A/B of the fused predict (PHD_FUSE_PREDICT) at config 3, plus config 2 (always fused)
set -u
mkdir -p gpurun_out/fab
for f in 0 1 0 1; do
  PHD_FUSE_PREDICT=$f timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/fab/b3_$f.json 2> gpurun_out/fab/b3_$f.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/fab/b3_$f.json'));print('c3 fuse $f:', d['value'], 'steps/s; ms/step', d['ms_per_step'], 'update ms', d['roofline']['avg_kernel_ms'])"
done
timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline > gpurun_out/fab/b2.json 2> gpurun_out/fab/b2.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/fab/b2.json'));print('c2:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
