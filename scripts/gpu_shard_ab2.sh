#!/bin/bash
# Sharded-step overhead, alternating A/B: libphdslam_base.so (A) vs
# libphdslam.so (B), emulated world 8 at config 3 and config 4; then the
# kernel stats of B's emulated world-8 step.
# usage: scripts/gpu_shard_ab2.sh <tag> [reps]
set -u
OUT=gpurun_out/${1:-shab}
mkdir -p $OUT
REPO=$(pwd)
for rep in $(seq 1 ${2:-2}); do
  for cfg in 3 4; do
    for v in A B; do
      if [ $v = A ]; then LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam_base.so; else LIB=$REPO/cuda-phdslam_amd/phdslam/libphdslam.so; fi
      PHDSLAM_LIB=$LIB timeout -k 10 300 python scripts/shard_overhead.py --config $cfg --world 8 --steps 300 > $OUT/ovh_c${cfg}_${v}_$rep.txt 2>&1 || { tail -20 $OUT/ovh_c${cfg}_${v}_$rep.txt; exit 1; }
      echo "c$cfg $v rep $rep: $(tail -1 $OUT/ovh_c${cfg}_${v}_$rep.txt | cut -c1-140)"
    done
  done
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp_w8 -o run -- python3 $REPO/scripts/shard_overhead.py --config 3 --world 8 --steps 100 > $REPO/$OUT/rp_w8.log 2>&1) || { tail -20 $OUT/rp_w8.log; exit 1; }
f=$(find $OUT/rp_w8 -name '*kernel_stats.csv' | head -1)
cp $f $OUT/w8_kernel_stats.csv
python3 - $f <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(x['Name'][:60].ljust(60), x['Calls'].rjust(6), '%9.1f' % (float(x['AverageNs']) / 1e3))
PY
