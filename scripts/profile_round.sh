#!/bin/bash
# Bench lines + rocprofv3 kernel stats (+ PMC traffic) for configs 2 and 3.
# Writes gpurun_out/prof_<tag>/{c<N>_bench.json,c<N>_kernel_stats.csv}; copy them to profiles/.
# usage: scripts/profile_round.sh <tag> [pmc]
set -u
TAG=$1
REPO=$(pwd)
OUT=$REPO/gpurun_out/prof_$TAG
mkdir -p "$OUT"
for CFG in 2 3; do
  timeout -k 10 300 python3 bench.py --config $CFG > "$OUT/c${CFG}_bench.json" 2> "$OUT/c${CFG}_bench.err" || exit $?
  cat "$OUT/c${CFG}_bench.json"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/rp_c$CFG" -o run -- python3 "$REPO/bench.py" --config $CFG --steps 200 --warmup 20 --no-cpu-baseline \
      > "$OUT/rp_c$CFG.log" 2>&1) || exit $?
  find "$OUT/rp_c$CFG" -name '*kernel_stats.csv' -exec cp {} "$OUT/c${CFG}_kernel_stats.csv" \;
  head -4 "$OUT/c${CFG}_kernel_stats.csv"
done
if [ "${2:-}" = pmc ]; then
  for CFG in 2 3; do bash scripts/pmc_traffic.sh $CFG || exit $?; done
fi
