#!/bin/bash
# round 3 checkpoint: full GPU suite + smoke + PMC + bench/kernel stats (gpu_final2.sh),
# then the sequence-mode line and the config-5 per-GPU line (8192 particles = 65536 / 8)
set -u
TAG=${1:-r03mid}
bash scripts/gpu_final2.sh $TAG || exit $?
OUT=gpurun_out/$TAG
timeout -k 10 300 python bench.py --config 3 --mode sequence --no-cpu-baseline > $OUT/c3_sequence_bench.json 2> $OUT/c3_sequence_bench.err || exit $?
cat $OUT/c3_sequence_bench.json
timeout -k 10 400 python bench.py --config 5 --particles 8192 --steps 50 --warmup 5 > $OUT/c5_pergpu_bench.json 2> $OUT/c5_pergpu_bench.err || exit $?
cat $OUT/c5_pergpu_bench.json
