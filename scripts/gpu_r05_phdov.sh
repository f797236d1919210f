#!/bin/bash
# split PHD step: the resample beside part C (config 4 / 5 per GPU, config 2)
set -u
T=${1:-r05ov}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "overlapped_resample or chunked_remap or fused_normalize_resample or bench_configuration" > $OUT/pytest.log 2>&1 \
  || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-config4-model "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'slow', d['config']['slow_paths'])"
}
b c4_pergpu --config 4 --particles 4096 --steps 300 || exit 1
b c5_pergpu --config 5 --particles 8192 --steps 100 || exit 1
b c2 --config 2 --steps 400 || exit 1
b c3 --steps 400 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o c4 -- python3 bench.py --no-cpu-baseline --no-config4-model --config 4 --particles 4096 --steps 200 > $OUT/prof_c4.log 2>&1 || { tail -5 $OUT/prof_c4.log; exit 1; }
f=$(find $OUT/prof_c4 -name '*kernel_stats.csv' | head -1); python3 -c "
import csv,sys
for r in list(csv.DictReader(open('$f')))[:6]: print('  %-40s %6s %8.1f us'%(r['Name'][:40],r['Calls'],float(r['AverageNs'])/1e3))"
