#!/bin/bash
# wave-per-particle kernel: parity tests, then bench lines for configs 3 and 2
set -u
OUT=gpurun_out/${1:-wave}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ${2:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in 3 2; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $OUT/b$c.json 2> $OUT/b$c.err || { cat $OUT/b$c.err | tail -5; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/b$c.json'));print('config $c', d['value'], 'steps/s, update', d['roofline']['avg_kernel_ms'], 'ms', d['config']['update_threads'], d['config']['update_lds_bytes'], d['config']['update_resident_workgroups'])"
done
exit 0
