#!/bin/bash
# bench.py's short-run sensitivity: 20 timed steps after 5 / 100 warm-up steps,
# 200 after 5, and 20 after 5 with a compute burst before (PHD_BENCH_SPIN)
for a in "20 5 0" "20 100 0" "20 5 40" "200 5 0" "20 5 0" "20 100 0" "20 5 40" "200 5 0"; do
  set -- $a
  if [ $3 = 0 ]; then SP=; else SP=$3; fi
  PHD_BENCH_SPIN=$SP timeout -k 10 200 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-config4-model > gpurun_out/w_$1_$2_$3.json 2>/dev/null && python3 -c "import json; d=json.load(open('gpurun_out/w_$1_$2_$3.json')); print('steps $1 warmup $2 spin $3:', d['value'])" || exit 1
done
