#!/bin/bash
# GPU parity suite + smoke on the current tree (round-end evidence shape).
# usage: scripts/gpu_tests.sh <tag> [pytest -k expression]
set -u
OUT=gpurun_out/${1:-tests}
mkdir -p $OUT
K=${2:-}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
