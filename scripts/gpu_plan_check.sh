#!/bin/bash
# GPU check of the sharded plan: full GPU parity suite, the sharded-step
# overhead at config 2 and 3 (world 8, emulated collectives), and a kernel
# trace of the config-3 run.
set -u
REPO=$(pwd)
mkdir -p gpurun_out/rp_plan
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/shard_overhead.py --config 2 --world 8 || exit $?
timeout -k 10 150 python scripts/shard_overhead.py --config 3 --world 8 --steps 60 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$REPO/gpurun_out/rp_plan" -o run -- python3 "$REPO/scripts/shard_overhead.py" --config 3 --world 8 --steps 40 \
    > "$REPO/gpurun_out/rp_plan/log.txt" 2>&1) || exit $?
cut -d, -f1-4 gpurun_out/rp_plan/run_kernel_stats.csv | cut -c1-150
