#!/bin/bash
# rocprofv3 kernel stats of the config-N bench: gpurun_out/<tag>/c<N>_kernel_stats.csv
set -u
T=${1:-kst}; C=${2:-3}
REPO=$(pwd)
OUT=$REPO/gpurun_out/$T
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rp_c$C -o run -- python3 $REPO/bench.py --config $C --steps 100 --warmup 10 --no-cpu-baseline > $OUT/rp_c$C.log 2>&1) || { tail -5 $OUT/rp_c$C.log; exit 1; }
find $OUT/rp_c$C -name '*kernel_stats.csv' -exec cp {} $OUT/c${C}_kernel_stats.csv \;
python3 - "$OUT/c${C}_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg_us {float(r['AverageNs'])/1e3:9.2f} pct {float(r['Percentage']):6.2f}")
PY
grep -v amdgpu.ids $OUT/rp_c$C.log | tail -1 | cut -c1-200
