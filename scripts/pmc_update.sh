#!/bin/bash
# PMC passes over the fused update (separate passes, --kernel-trace off; counters per guide §rocprofv3).
# usage: scripts/pmc_update.sh <config> <pass-name> <counters...>
set -u
CFG=$1; NAME=$2; shift 2
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc_c${CFG}_$NAME
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT" -o run -- python3 "$REPO/bench.py" --config "$CFG" --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/log.txt" 2>&1
