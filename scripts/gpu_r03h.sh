#!/bin/bash
set -u
OUT=gpurun_out/${1:-r03h}
mkdir -p $OUT
bash scripts/gpu_ab.sh ${1:-r03h}_ab 3 PHD_MERGE_CELL=0 || exit 1
timeout -k 10 1200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread -p no:cacheprovider \
  -k "bench_configuration or cphd_update_matches or update_matches_oracle or merge or fallback or overflow or tiny or ragged or range or labels or config5 or bearing" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; exit $rc
