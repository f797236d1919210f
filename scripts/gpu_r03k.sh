#!/bin/bash
# round 3: wave-uniform merge walk with scan listing — A/B, stamps, merge/update parity
set -u
OUT=gpurun_out/${1:-r03k}
mkdir -p $OUT
bash scripts/gpu_ab.sh ${1:-r03k} 3 || exit $?
timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/stamps_c3.txt 2>&1 || exit $?
grep -E "cull|lfmis|emit" $OUT/stamps_c3.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "merge or update or cphd" > $OUT/pytest_parity.log 2>&1
rc=$?; tail -3 $OUT/pytest_parity.log; exit $rc
