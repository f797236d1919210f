#!/bin/bash
# sharded-step overhead (world 8, config 3, emulated transport) without and with migration
set -u
OUT=gpurun_out/${1:-shard_mig}
mkdir -p $OUT
for s in 0 -0.002 0.002 -0.02; do
  timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 100 --skew=$s > $OUT/ovh_$s.txt 2>&1 || { tail -3 $OUT/ovh_$s.txt; exit 1; }
  echo "skew $s: $(tail -1 $OUT/ovh_$s.txt)"
done
