#!/bin/bash
# round 3: merge-walk divergence stamps at config 3
set -u
OUT=gpurun_out/${1:-r03j}
mkdir -p $OUT
timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/stamps_c3.txt 2>&1
rc=$?; cat $OUT/stamps_c3.txt; exit $rc
