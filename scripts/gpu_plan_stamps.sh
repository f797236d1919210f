#!/bin/bash
# bench at config 3 (sampled timing events), the sharded plan's phase stamps
# at an emulated world 8 (configs 3 and 4) and the sharded-step overhead.
# usage: scripts/gpu_plan_stamps.sh <tag>
set -u
OUT=gpurun_out/${1:-pstamps}
mkdir -p $OUT
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 200 > $OUT/c3.json 2> $OUT/c3.err || { tail -20 $OUT/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3.json'));print('c3:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'timed', d['roofline']['timed_updates'])"
for c in 3 4; do
  timeout -k 10 300 python scripts/plan_stamps.py --config $c --world 8 --plans 50 > $OUT/stamps_c$c.txt 2>&1 || { tail -20 $OUT/stamps_c$c.txt; exit 1; }
  cat $OUT/stamps_c$c.txt
done
timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 200 > $OUT/ovh_c3.txt 2>&1 || { tail -20 $OUT/ovh_c3.txt; exit 1; }
tail -1 $OUT/ovh_c3.txt
