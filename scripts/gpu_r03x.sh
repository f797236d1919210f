#!/bin/bash
# round 3: part C without scratch spills (packed batched scans) — A/B, traffic, merge parity
set -u
OUT=gpurun_out/${1:-r03x}
mkdir -p $OUT
bash scripts/gpu_ab.sh ${1:-r03x} 3 || exit $?
bash scripts/pmc_traffic.sh 3 > $OUT/traffic.log 2>&1 || { tail -3 $OUT/traffic.log; exit 1; }
tail -12 $OUT/traffic.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "merge or update or cphd" > $OUT/pytest_parity.log 2>&1
rc=$?; tail -3 $OUT/pytest_parity.log; exit $rc
