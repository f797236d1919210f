#!/bin/bash
# round 3: EAP decision-round timing at config 3
set -u
OUT=gpurun_out/${1:-r03p}
mkdir -p $OUT
PHD_EAP_DEBUG=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 500 --timeout-method thread -p no:cacheprovider -s \
  -k "expected_map_config3" > $OUT/pytest_eap.log 2>&1
rc=$?; grep -E "eap" $OUT/pytest_eap.log | head -60; tail -2 $OUT/pytest_eap.log; exit $rc
