#!/bin/bash
# A/B of update variants at config 3: libphdslam.so against libphdslam_v<tag>.so
# for each tag given, alternating, rocprofv3 kernel stats of bench.py (update
# launches), then the bench-configuration parity test on each variant.
# usage: scripts/gpu_variants.sh <out-tag> <reps> <variant-tag>...
set -u
OUT=gpurun_out/$1; REPS=$2; shift 2
mkdir -p $OUT
REPO=$(pwd)
for rep in $(seq 1 $REPS); do
  for v in main "$@"; do
    if [ $v = main ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_v$v.so; fi
    (cd /tmp && export TMPDIR=/tmp && PHDSLAM_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp_${v}_$rep -o run -- python3 $REPO/bench.py --config 3 --no-cpu-baseline --steps 200 --warmup 20 > $REPO/$OUT/b_${v}_$rep.json 2> $REPO/$OUT/b_${v}_$rep.err) || { tail -5 $OUT/b_${v}_$rep.err; exit 1; }
    f=$(find $OUT/rp_${v}_$rep -name '*kernel_stats.csv' | head -1)
    python3 - "$f" $v $rep $OUT/b_${v}_$rep.json <<'PY'
import csv, sys, json
rows = list(csv.DictReader(open(sys.argv[1])))
out = []
for r in rows:
    nm = r["Name"]
    if any(k in nm for k in ("k_update_", "k_cphd_terms")):
        out.append(f"{nm.split('(')[0].replace('phd::k_','')}={float(r['AverageNs'])/1e3:.1f}us")
d = json.load(open(sys.argv[4]))
print(sys.argv[2], "rep", sys.argv[3], d["value"], "steps/s", d["config"].get("update_lds_bytes"), d["config"].get("update_resident_workgroups"), " ".join(sorted(out)))
PY
  done
done
for v in "$@"; do
  PHDSLAM_LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_v$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "cphd_update_bench_configuration or test_cphd_update_matches_oracle" > $OUT/parity_$v.log 2>&1 || { tail -30 $OUT/parity_$v.log; exit 1; }
  echo "parity $v: $(tail -1 $OUT/parity_$v.log)"
done
