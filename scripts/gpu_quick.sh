#!/bin/bash
# Quick GPU iteration: parity tests (optionally filtered), bench lines, phase stamps.
# usage: scripts/gpu_quick.sh "<pytest -k expr or empty>" "<configs>" [stamps]
set -u
mkdir -p gpurun_out
K=${1:-}
CFGS=${2:-"2 3"}
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -4 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
fi
for c in $CFGS; do
  timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > gpurun_out/b$c.json 2> gpurun_out/b$c.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/b$c.json'));print('config $c', d['value'], 'steps/s, update', d['roofline']['avg_kernel_ms'], 'ms')"
done
if [ "${3:-}" = stamps ]; then
  for c in $CFGS; do
    timeout -k 10 200 python scripts/phase_stamps.py --config $c > gpurun_out/st$c.log 2>&1 || exit $?
  done
fi
exit 0
