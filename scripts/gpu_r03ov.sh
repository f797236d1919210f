#!/bin/bash
# round 3: normalise + resample beside part C (side stream) — A/B, then the full GPU suite
set -u
OUT=gpurun_out/${1:-r03ov}
mkdir -p $OUT
bash scripts/gpu_ab.sh ${1:-r03ov} 3 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; exit $rc
