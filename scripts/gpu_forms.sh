#!/bin/bash
# PHD update forms (1 fused, 2 split) x workgroup sizes at a config's per-GPU shape
# usage: scripts/gpu_forms.sh <tag> <config> [particles]
set -u
OUT=gpurun_out/${1:-forms}
CFG=${2:-4}
NP=${3:-0}
mkdir -p $OUT
extra=""; [ "$NP" != 0 ] && extra="--particles $NP"
for spec in "0 0" "1 256" "1 512" "2 256" "2 512"; do
  set -- $spec
  timeout -k 10 240 python bench.py --config $CFG $extra --form $1 --threads $2 --no-cpu-baseline --steps 60 --warmup 10 > $OUT/c${CFG}_f$1_t$2.json 2> $OUT/c${CFG}_f$1_t$2.err || { tail -5 $OUT/c${CFG}_f$1_t$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c${CFG}_f$1_t$2.json'));c=d['config'];print('c$CFG form $1 threads $2:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], c['update_threads'], c['update_split'], c['update_resident_workgroups'])"
done
