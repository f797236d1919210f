#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration (known bytes per access width) -> gpurun_out/calib
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-calib}
mkdir -p $OUT
BIN=$GRAFT_REPO_ROOT/scripts/calib/calib_fetch
timeout -k 10 60 $BIN > $OUT/bytes.csv || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $BIN > $OUT/fetch.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $BIN > $OUT/write.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT && python3 scripts/calib/fetch_report.py $OUT > $OUT/fetch_calibration.json && cat $OUT/fetch_calibration.json
