#!/bin/bash
# quick confirmation of the committed tree: GPU tests, smoke, default bench lines
set -u
OUT=gpurun_out/${1:-confirm}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for c in 3 2; do
  timeout -k 10 300 python bench.py --config $c > $OUT/c${c}_bench.json 2> $OUT/c${c}_bench.err || exit $?
  python3 -c "import json;d=json.load(open('$OUT/c${c}_bench.json'));print('config $c:', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'])"
done
