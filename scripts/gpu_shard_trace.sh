#!/bin/bash
# Kernel timeline of the sharded step at an emulated world 8 (scripts/shard_overhead.py):
# the per-kernel stats and the raw trace, from which the per-step gaps between the
# sharded step's launches are read (scripts/trace_gaps.py).
# usage: scripts/gpu_shard_trace.sh <tag> [shard_overhead args]
set -u
OUT=gpurun_out/${1:-shard_trace}
shift
mkdir -p $OUT
REPO=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $REPO/$OUT/rp -o run -- python3 $REPO/scripts/shard_overhead.py --config 3 --world 8 --steps 100 "$@" > $REPO/$OUT/ovh.log 2>&1) || { tail -20 $OUT/ovh.log; exit 1; }
tail -1 $OUT/ovh.log
find $OUT/rp -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/rp -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/rp -name '*memory_copy_trace.csv' -exec cp {} $OUT/memory_copy_trace.csv \;
rm -rf $OUT/rp
cut -c1-150 $OUT/kernel_stats.csv
