#!/bin/bash
# The wave-per-particle form (threads 64) against the workgroup form (auto
# threads) at configs 2, 3 and 5 (per GPU: 8192 particles), bench lines only.
# usage: scripts/gpu_wave_vs_wg.sh <tag>
set -u
OUT=gpurun_out/${1:-wavewg}
mkdir -p $OUT
for spec in "3 0 0" "3 64 0" "2 0 0" "2 64 0" "5 0 8192" "5 64 8192"; do
  set -- $spec
  CFG=$1; TH=$2; NP=$3
  extra=""; [ "$NP" != 0 ] && extra="--particles $NP"
  timeout -k 10 240 python bench.py --config $CFG --threads $TH $extra --no-cpu-baseline --steps 100 --warmup 10 \
      > $OUT/c${CFG}_t${TH}.json 2> $OUT/c${CFG}_t${TH}.err || { tail -5 $OUT/c${CFG}_t${TH}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c${CFG}_t${TH}.json'));print('c$CFG threads $TH:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], d['config']['update_threads'], d['config']['update_resident_workgroups'])"
done
