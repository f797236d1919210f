#!/bin/bash
# A/B of the wave-priority ramp of the update workgroups (PHD_UPD_PRIO)
set -u
mkdir -p gpurun_out/prio
for c in 3; do
for p in 0 40 190 200 210 0 40 200; do
  PHD_UPD_PRIO=$p timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 300 --warmup 30 > gpurun_out/prio/b${c}_$p.json 2> gpurun_out/prio/b${c}_$p.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/prio/b${c}_$p.json'));print('c$c prio $p:', d['value'], 'steps/s; ms/step', d['ms_per_step'], 'update ms', d['roofline']['avg_kernel_ms'])"
done
done
