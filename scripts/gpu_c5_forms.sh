#!/bin/bash
# config 5 per GPU (8192 x 1024 x 128): the split update at 256 / 512 / 1024
# threads and the auto choice, then the kernel stats of the auto choice.
# usage: scripts/gpu_c5_forms.sh <tag>
set -u
OUT=gpurun_out/${1:-c5forms}
mkdir -p $OUT
REPO=$(pwd)
for args in "--form 2 --threads 256" "--form 2 --threads 512" "--form 2 --threads 1024" ""; do
  tag=$(echo "x$args" | tr -d ' -')
  timeout -k 10 300 python bench.py --config 5 --particles 8192 --steps 40 --warmup 5 --no-cpu-baseline $args > $OUT/c5_$tag.json 2> $OUT/c5_$tag.err || { tail -5 $OUT/c5_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/c5_$tag.json'));c=d['config'];print('$args', d['value'], c.get('update_threads'), c.get('update_split'), c.get('update_resident_workgroups'), c.get('update_lds_bytes'))"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $REPO/$OUT/rp -o run -- python3 $REPO/bench.py --config 5 --particles 8192 --steps 20 --warmup 5 --no-cpu-baseline > $REPO/$OUT/rp.log 2>&1) || { tail -5 $OUT/rp.log; exit 1; }
find $OUT/rp -name '*kernel_stats.csv' -exec cp {} $OUT/c5_kernel_stats.csv \;
rm -rf $OUT/rp
cut -d, -f1-4 $OUT/c5_kernel_stats.csv | head -8
