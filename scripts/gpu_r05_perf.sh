#!/bin/bash
# round-5 performance evidence: bench lines of every config shape, the sharded
# overhead at emulated world 8, part C / part A phase stamps with births,
# kernel stats of the config-3 step.
set -u
OUT=gpurun_out/${1:-r05p}
mkdir -p $OUT
b() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || { tail -5 $OUT/$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));print('$name', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'frac', d['roofline']['frac'], 'thr/lds/res', d['config']['update_threads'], d['config']['update_lds_bytes'], d['config']['update_resident_workgroups'], 'split', d['config']['update_split'], 'slow', d['config']['slow_paths'], 'cpu', d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('cores'))"
}
b c3 --steps 400 || exit 1
b c3_nobirths --births 0 --no-cpu-baseline --steps 400 || exit 1
b c2 --config 2 --no-cpu-baseline --steps 400 || exit 1
b c4_pergpu --config 4 --particles 4096 --steps 300 || exit 1
b c5_pergpu --config 5 --particles 8192 --steps 100 || exit 1
timeout -k 10 300 python scripts/shard_overhead.py --config 3 --world 8 --steps 300 > $OUT/shard_overhead_c3_w8.txt 2>&1 || { tail -5 $OUT/shard_overhead_c3_w8.txt; exit 1; }
cat $OUT/shard_overhead_c3_w8.txt
timeout -k 10 300 python scripts/shard_overhead.py --config 4 --world 8 --steps 300 > $OUT/shard_overhead_c4_w8.txt 2>&1 || { tail -5 $OUT/shard_overhead_c4_w8.txt; exit 1; }
cat $OUT/shard_overhead_c4_w8.txt
timeout -k 10 300 python scripts/phase_stamps.py --config 3 > $OUT/stamps_c3_partC.txt 2>&1 || { tail -5 $OUT/stamps_c3_partC.txt; exit 1; }
timeout -k 10 300 python scripts/phase_stamps.py --config 3 --part A > $OUT/stamps_c3_partA.txt 2>&1 || { tail -5 $OUT/stamps_c3_partA.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 -- python3 bench.py --steps 100 --no-cpu-baseline > $OUT/prof_c3.json 2> $OUT/prof_c3.err || { tail -5 $OUT/prof_c3.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
