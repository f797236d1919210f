#!/bin/bash
# event-scope A/B: config-3 bench alternating over two libraries, then the
# sharded-step overhead at an emulated world 8 under each, then a kernel trace
# of the fused step under the first.
# usage: scripts/gpu_ev_ab.sh <tag> <reps> <libA> <libB>
set -u
OUT=gpurun_out/${1:-evab}
REPS=$2; A=$3; B=$4
mkdir -p $OUT
bash scripts/gpu_abn.sh ${1:-evab} $REPS $A $B || exit $?
for v in $A $B; do
  PHDSLAM_LIB=$PWD/cuda-phdslam_amd/phdslam/$v timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 200 > $OUT/ovh_$v.txt 2>&1 || { tail -20 $OUT/ovh_$v.txt; exit 1; }
  echo "$v: $(tail -1 $OUT/ovh_$v.txt)"
done
REPO=$(pwd)
(cd /tmp && export TMPDIR=/tmp && PHDSLAM_LIB=$REPO/cuda-phdslam_amd/phdslam/$A timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp -o run -- python3 $REPO/bench.py --config 3 --no-cpu-baseline --steps 100 --warmup 10 > $REPO/$OUT/rp.log 2>&1) || { tail -20 $OUT/rp.log; exit 1; }
find $OUT/rp -name '*kernel_trace.csv' -exec cp {} $OUT/kernel_trace.csv \;
find $OUT/rp -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
rm -rf $OUT/rp
