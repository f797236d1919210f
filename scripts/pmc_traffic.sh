#!/bin/bash
# HBM traffic of the fused update per the MI355X guide (§HBM): FETCH_SIZE and
# WRITE_SIZE in separate --pmc passes (they do not fit one pass), same bench
# command, then scripts/pmc_traffic.py applies the gfx950 correction.
# usage: scripts/pmc_traffic.sh <config>
set -u
CFG=$1
REPO=$(pwd)
OUT=$REPO/gpurun_out/traffic_c$CFG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$OUT/$C" -o run -- python3 "$REPO/bench.py" --config "$CFG" --steps 20 --warmup 2 --no-cpu-baseline > "$OUT/$C.log" 2>&1 || exit $?
done
cd "$REPO" && python3 scripts/pmc_traffic.py "$CFG" "$OUT"
