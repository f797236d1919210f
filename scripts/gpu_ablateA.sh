#!/bin/bash
# Part A timing ablations at config 3 (PHD_XK 11 / 12 / 13, libphdslam_k<x>.so,
# results wrong by design) against the shipped library, alternating, with
# per-kernel durations from rocprofv3 kernel stats.
# usage: scripts/gpu_ablateA.sh <tag> [reps]
set -u
OUT=gpurun_out/${1:-ablA}
mkdir -p $OUT
REPO=$(pwd)
for rep in $(seq 1 ${2:-2}); do
  for v in base 11 12 13; do
    if [ $v = base ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_k$v.so; fi
    (cd /tmp && export TMPDIR=/tmp && PHDSLAM_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp_${v}_$rep -o run -- python3 $REPO/bench.py --config 3 --no-cpu-baseline --steps 100 --warmup 10 > $REPO/$OUT/b_${v}_$rep.json 2> $REPO/$OUT/b_${v}_$rep.err) || { tail -5 $OUT/b_${v}_$rep.err; exit 1; }
    f=$(find $OUT/rp_${v}_$rep -name '*kernel_stats.csv' | head -1)
    python3 - "$f" $v $rep <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    nm = r["Name"]
    if any(k in nm for k in ("k_update_cphd", "k_cphd_terms")):
        out.append(f"{nm.split('(')[0].replace('phd::k_','')}={float(r['AverageNs'])/1e3:.1f}us")
print(sys.argv[2], "rep", sys.argv[3], " ".join(out))
PY
  done
done
