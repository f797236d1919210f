#!/bin/bash
# A/B (alternating) of the particle order of the CPHD terms / part C launches
# (PHD_UPD_ORDER: 0 identity, 1 XCD-preserving last-written-first), then the CPHD parity tests
set -u
mkdir -p gpurun_out/oab
i=0
for o in 0 1 0 1 0 1; do
  i=$((i+1))
  PHD_UPD_ORDER=$o timeout -k 10 200 python bench.py --config 3 --no-cpu-baseline --steps 400 --warmup 40 > gpurun_out/oab/b_${o}_$i.json 2> gpurun_out/oab/b_${o}_$i.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/oab/b_${o}_$i.json'));print('order $o:', d['value'], 'steps/s; ms/step', d['ms_per_step'], 'update ms', d['roofline']['avg_kernel_ms'])"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "cphd or shard or step" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/oab/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/oab/pytest.log; exit $rc
