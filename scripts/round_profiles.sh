#!/bin/bash
# Round-end evidence: bench lines + kernel stats + PMC traffic for configs 2 and 3
# (profile_round.sh), then the sharded-step overhead (world 8, emulated
# collectives) with a kernel trace of the config-3 run.
set -u
TAG=$1
REPO=$(pwd)
bash scripts/profile_round.sh "$TAG" pmc || exit $?
OUT=$REPO/gpurun_out/prof_$TAG
timeout -k 10 150 python scripts/shard_overhead.py --config 2 --world 8 > "$OUT/shard_c2_w8.txt" 2>&1 || exit $?
timeout -k 10 200 python scripts/shard_overhead.py --config 3 --world 8 --steps 60 > "$OUT/shard_c3_w8.txt" 2>&1 || exit $?
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
    -d "$OUT/rp_shard_c3" -o run -- python3 "$REPO/scripts/shard_overhead.py" --config 3 --world 8 --steps 40 \
    > "$OUT/rp_shard_c3.log" 2>&1) || exit $?
find "$OUT/rp_shard_c3" -name '*kernel_stats.csv' -exec cp {} "$OUT/shard_c3_w8_kernel_stats.csv" \;
tail -1 "$OUT/shard_c2_w8.txt"; tail -1 "$OUT/shard_c3_w8.txt"
