#!/bin/bash
# stall / fetch counters of the config-3 update kernels (one PMC pass each)
# usage: [PASSES='name:C1 C2 ..' ...] scripts/gpu_icache.sh <tag>
set -u
T=${1:-icache}
REPO=$(pwd)
OUT=$REPO/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
if [ -n "${PASSES:-}" ]; then LIST=("$PASSES"); else
  LIST=("ic:SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "wait:SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"); fi
for P in "${LIST[@]}"; do
  NAME=${P%%:*}; CNT=${P#*:}
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/$NAME" -o run -- python3 "$REPO/bench.py" --config 3 --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/$NAME.log" 2>&1 || { tail -3 "$OUT/$NAME.log"; exit 1; }
done
cd "$REPO" && python3 - "$OUT" <<'PY'
import sys
sys.path.insert(0, "scripts")
from pmc_report import counters
acc = counters(sys.argv[1])
for k, d in sorted(acc.items()):
    print(k, {c: round(v) for c, v in sorted(d.items())})
PY
