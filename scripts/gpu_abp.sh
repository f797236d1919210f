#!/bin/bash
# alternating A/B (libphdslam_base.so vs libphdslam.so, config 3) + the update / merge parity tests
set -u
OUT=gpurun_out/${1:-abp}
mkdir -p $OUT
bash scripts/gpu_ab.sh ${1:-abp} ${2:-3} || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "merge or update or cphd" > $OUT/pytest_parity.log 2>&1
rc=$?; tail -2 $OUT/pytest_parity.log; exit $rc
