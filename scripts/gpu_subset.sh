#!/bin/bash
# A pytest -m gpu subset (-k expression) + smoke + the default bench line.
# usage: scripts/gpu_subset.sh <tag> "<k-expr>"
set -u
OUT=gpurun_out/${1:-subset}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -p no:cacheprovider -k "$2" > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_c3.json'));print('c3', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'cpu', d['cpu_baseline'].get('value'), d['cpu_baseline'].get('cores'))"
