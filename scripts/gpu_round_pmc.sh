#!/bin/bash
# PMC passes (HBM traffic, instruction counts) + kernel stats of the update for one config
# usage: [PARTICLES=n] scripts/gpu_round_pmc.sh <tag> <config>
# (PARTICLES: a per-GPU shape other than the config's default; the reports are
# then named pmc_c<C>_n<n>.json / traffic_c<C>_n<n>.json)
set -u
T=${1:-pmc}; C=${2:-3}
PARGS=${PARTICLES:+--particles $PARTICLES}
REPO=$(pwd)
OUT=$REPO/gpurun_out/$T
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for P in FETCH_SIZE WRITE_SIZE "util:SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  NAME=${P%%:*}; CNT=${P#*:}
  timeout -s KILL 120 rocprofv3 --pmc $CNT --output-format csv -d "$OUT/$NAME" -o run -- python3 "$REPO/bench.py" --config "$C" $PARGS --steps 20 --warmup 2 --no-cpu-baseline --no-config4-model > "$OUT/$NAME.log" 2>&1 || { tail -3 "$OUT/$NAME.log"; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 "$REPO/bench.py" --config "$C" $PARGS --steps 100 --warmup 10 --no-cpu-baseline --no-config4-model > "$OUT/stats.log" 2>&1 || { tail -3 "$OUT/stats.log"; exit 1; }
find "$OUT/stats" -name '*kernel_stats.csv' -exec cp {} "$OUT/c${C}_kernel_stats.csv" \;
cd "$REPO" && python3 scripts/pmc_report.py "$C" "$OUT" ${PARTICLES:-}
