#!/bin/bash
# A/B of the wave-priority tail (PHD_UPD_PRIO) with the last-written-first part C order
set -u
mkdir -p gpurun_out/prio2
for p in ${PRIOS:-40 25 55 40 25 55}; do
  PHD_UPD_PRIO=$p timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 400 --warmup 40 > gpurun_out/prio2/b_$p.json 2> gpurun_out/prio2/b_$p.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/prio2/b_$p.json'));print('prio $p:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
done
