#!/bin/bash
# Round-4 closing evidence on the final tree: scripts/gpu_final4.sh (GPU suite +
# smoke, PMC passes, bench lines + kernel stats of configs 2 / 3, per-GPU lines
# of configs 4 / 5), then the sequence-mode line, the sharded step at world 1
# over RCCL (Python) and from the C++ group host, and the sharded-step overhead
# at an emulated world 8 (configs 3 and 4).
# usage: scripts/gpu_final4b.sh <tag>
set -u
TAG=${1:-r04fin}
OUT=gpurun_out/$TAG
mkdir -p $OUT
bash scripts/gpu_final4.sh $TAG || exit $?
timeout -k 10 300 python bench.py --config 3 --mode sequence --no-cpu-baseline --steps 200 > $OUT/c3_sequence_bench.json 2> $OUT/c3_sequence.err || { tail -20 $OUT/c3_sequence.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3_sequence_bench.json'));print('sequence:', d['value'], d.get('slow_paths'))"
timeout -k 10 300 python bench.py --config 3 --force-sharded --no-cpu-baseline --steps 200 --warmup 20 > $OUT/c3_rccl_w1.json 2> $OUT/c3_rccl_w1.err || { tail -20 $OUT/c3_rccl_w1.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3_rccl_w1.json'));print('rccl world 1:', d['value'], d['config']['parallelism'])"
timeout -k 10 300 cuda-phdslam_amd/phdslam/phdslam_run --synth 3 --gpus 1 --replay --steps 200 > $OUT/c3_group_w1.json 2> $OUT/c3_group_w1.err || { tail -20 $OUT/c3_group_w1.err; exit 1; }
cat $OUT/c3_group_w1.json
for c in 3 4; do
  timeout -k 10 300 python scripts/shard_overhead.py --config $c --world 8 --steps 200 > $OUT/ovh_c$c.txt 2>&1 || { tail -20 $OUT/ovh_c$c.txt; exit 1; }
  echo "c$c: $(tail -1 $OUT/ovh_c$c.txt)"
done
