#!/bin/bash
# GPU check of the sharded-step path: resample/step parity tests, then a
# kernel-trace profile of scripts/shard_overhead.py (world 8, config 2).
set -u
REPO=$(pwd)
mkdir -p gpurun_out/rp_shard
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "shard or resample or step or sequence" > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$REPO/gpurun_out/rp_shard" -o run -- python3 "$REPO/scripts/shard_overhead.py" --config 2 --world 8 \
    > "$REPO/gpurun_out/rp_shard/log.txt" 2>&1) || exit $?
timeout -k 10 100 python scripts/shard_overhead.py --config 2 --world 8 2>&1 | grep fused
