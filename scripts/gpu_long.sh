#!/bin/bash
# long runs at config 3: 2000 timed steps in replay and in sequence mode (a
# fresh measurement set every step), with the slow-path counters of every
# timed step
# usage: scripts/gpu_long.sh <tag>
set -u
OUT=gpurun_out/${1:-long}
mkdir -p $OUT
for mode in replay sequence; do
  timeout -k 10 300 python bench.py --config 3 --mode $mode --no-cpu-baseline --steps 2000 --warmup 20 > $OUT/c3_${mode}_2000.json 2> $OUT/c3_${mode}.err || { tail -20 $OUT/c3_${mode}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c3_${mode}_2000.json'));print('$mode', d['value'], d['ms_per_step'], d['config']['slow_paths'], d['roofline']['timed_updates'], d['roofline']['avg_kernel_ms'])"
done
