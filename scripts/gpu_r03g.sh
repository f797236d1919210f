#!/bin/bash
# round 3: production-occupancy phase costs of part C (ablation builds, PHD_XK), old merge
set -u
OUT=gpurun_out/${1:-r03g}
mkdir -p $OUT
for x in base 3 4 6 7 8 9 base; do
  if [ $x = base ]; then LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam.so; else LIB=$PWD/cuda-phdslam_amd/phdslam/libphdslam_k$x.so; fi
  PHD_MERGE_CELL=${CELL:-0} PHDSLAM_LIB=$LIB timeout -k 10 120 python bench.py --config 3 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/b_$x.json 2> $OUT/b_$x.err
  python3 -c "import json;d=json.load(open('$OUT/b_$x.json'));print('$x', d['value'], 'steps/s, update', d['roofline']['avg_kernel_ms'], 'ms')" 2>/dev/null || { echo "$x failed"; tail -2 $OUT/b_$x.err; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 1
find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv" -exec head -8 {} \;
exit 0
