#!/bin/bash
# GPU suite + replay / sequence config-3 bench lines (slow-path counters)
set -u
T=${1:-r05w}
bash scripts/gpu_tests.sh $T || exit $?
OUT=gpurun_out/$T
timeout -k 10 300 python bench.py --steps 400 --no-cpu-baseline --no-config4-model > $OUT/c3.json 2> $OUT/c3.err || exit 1
timeout -k 10 300 python bench.py --mode sequence --steps 400 --no-cpu-baseline --no-config4-model > $OUT/c3_seq.json 2> $OUT/c3_seq.err || exit 1
for f in c3 c3_seq; do
  python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', d['value'], d['roofline']['avg_kernel_ms'], d['config']['slow_paths'])"
done
