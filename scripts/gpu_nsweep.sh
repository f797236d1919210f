#!/bin/bash
# update-kernel time against the particle count at config 3 (round quantisation)
set -u
mkdir -p gpurun_out/nsw
for n in 1792 2048 3072 3584 4096 4608 5376; do
  timeout -k 10 200 python bench.py --config 3 --particles $n --no-cpu-baseline --steps 200 --warmup 20 > gpurun_out/nsw/b_$n.json 2> gpurun_out/nsw/b_$n.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/nsw/b_$n.json'));print('n $n:', d['value'], 'steps/s; ms/step', d['ms_per_step'], 'update ms', d['roofline']['avg_kernel_ms'])"
done
cd /tmp && export TMPDIR=/tmp
for n in 1792 3584 4096; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/nsw/p$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --particles $n --steps 50 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/nsw/p$n.log 2>&1 || exit $?
done
