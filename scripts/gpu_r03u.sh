#!/bin/bash
# round 3: persistent part C (A: PHD_PERSIST=1) vs the shipped launch (B), same library; parity under PHD_PERSIST
set -u
OUT=gpurun_out/${1:-r03u}
mkdir -p $OUT
bash scripts/gpu_ab.sh ${1:-r03u} 3 PHD_PERSIST=1 || exit $?
PHD_PERSIST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "bench_configuration or config3 or cphd_update" > $OUT/pytest_persist.log 2>&1
rc=$?; tail -3 $OUT/pytest_persist.log; exit $rc
