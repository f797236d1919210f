#!/bin/bash
# config 2: the automatic form against the forced fused / split forms
set -u
OUT=gpurun_out/${1:-c2forms}
mkdir -p $OUT
for f in 0 1 2 0; do
  timeout -k 10 200 python bench.py --config 2 --no-cpu-baseline --steps 400 --form $f > $OUT/c2_f$f.json 2> $OUT/c2_f$f.err || { tail -5 $OUT/c2_f$f.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c2_f$f.json'));print('form $f', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], d['config']['update_threads'], d['config']['update_lds_bytes'], d['config']['update_resident_workgroups'], 'split', d['config']['update_split'])"
done
