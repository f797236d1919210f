#!/bin/bash
# The sharded plan: parity tests of every sharded path (one-launch k_shard_plan,
# strata past the CDF's end, the C++ group host), the plan's own overhead at an
# emulated world 8 (config 3 and config 4, with and without migration), RCCL at
# world 1 (bench.py --force-sharded) with its kernel trace, and the C++ group
# host at world 1.
# usage: scripts/gpu_plan.sh <tag>
set -u
OUT=gpurun_out/${1:-plan}
mkdir -p $OUT
REPO=$(pwd)
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -k "shard or group" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for args in "--config 3" "--config 3 --skew 0.5" "--config 4" "--config 4 --skew 0.5"; do
  tag=$(echo $args | tr -d ' -')
  timeout -k 10 300 python scripts/shard_overhead.py $args --world 8 --steps 200 > $OUT/ovh_$tag.txt 2>&1 || { tail -20 $OUT/ovh_$tag.txt; exit 1; }
  echo "$args: $(tail -1 $OUT/ovh_$tag.txt)"
done
timeout -k 10 300 python bench.py --config 3 --force-sharded --no-cpu-baseline --steps 200 --warmup 20 > $OUT/c3_rccl_w1.json 2> $OUT/c3_rccl_w1.err || { tail -20 $OUT/c3_rccl_w1.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/c3_rccl_w1.json'));print('rccl world 1:', d['value'], d['config']['parallelism'])"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp_rccl -o run -- python3 $REPO/bench.py --config 3 --force-sharded --no-cpu-baseline --steps 100 --warmup 10 > $REPO/$OUT/rp_rccl.log 2>&1) || { tail -20 $OUT/rp_rccl.log; exit 1; }
find $OUT/rp_rccl -name '*kernel_stats.csv' -exec cp {} $OUT/c3_rccl_w1_kernel_stats.csv \;
timeout -k 10 300 cuda-phdslam_amd/phdslam/phdslam_run --synth 3 --gpus 1 --replay --steps 200 > $OUT/c3_group_w1.json 2> $OUT/c3_group_w1.err || { tail -20 $OUT/c3_group_w1.err; exit 1; }
cat $OUT/c3_group_w1.json
