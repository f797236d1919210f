#!/bin/bash
# Update launch times against the particle count at config 3 (rounds of
# resident workgroups: part C 1792 / part A 1536 slots at 256 threads):
# rocprofv3 kernel stats of bench.py --particles N for each N.
# usage: scripts/gpu_rounds.sh <tag> N1 N2 ...
set -u
TAG=$1; shift
REPO=$(pwd)
OUT=$REPO/gpurun_out/$TAG
mkdir -p "$OUT"
for NP in "$@"; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/rp_$NP" -o run -- python3 "$REPO/bench.py" --config 3 --particles $NP --steps 100 --warmup 10 \
      --no-cpu-baseline > "$OUT/b_$NP.json" 2> "$OUT/b_$NP.err") || { tail -5 "$OUT/b_$NP.err"; exit 1; }
  f=$(find "$OUT/rp_$NP" -name '*kernel_stats.csv' | head -1)
  cp "$f" "$OUT/stats_$NP.csv"
  python3 - "$OUT/stats_$NP.csv" $NP <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    nm = r["Name"]
    if any(k in nm for k in ("k_update_cphd", "k_cphd_terms", "k_predict", "k_rs_")):
        out.append(f"{nm.split('(')[0]}={float(r['AverageNs'])/1e3:.1f}us")
print("N", sys.argv[2], " ".join(out))
PY
done
