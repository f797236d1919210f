#!/bin/bash
# round 3: EAP by synchronous decision rounds — parity at every scale + config-3 timing
set -u
OUT=gpurun_out/${1:-r03o}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mixed.py tests/test_gpu_shim.py -x -q --timeout 500 --timeout-method thread -p no:cacheprovider -s \
  -k "expected_map or eap or recover" > $OUT/pytest_eap.log 2>&1
rc=$?; tail -3 $OUT/pytest_eap.log; grep -E "eap config" $OUT/pytest_eap.log; exit $rc
