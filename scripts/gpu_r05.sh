#!/bin/bash
# round-5 evidence: GPU suite + smoke, config-3 bench (births on, off), kernel stats
set -u
OUT=gpurun_out/${1:-r05}
mkdir -p $OUT
bash scripts/gpu_tests.sh ${1:-r05} ${2:-} || exit $?
timeout -k 10 400 python bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { tail -5 $OUT/bench_c3.err; exit 1; }
timeout -k 10 400 python bench.py --births 0 --no-cpu-baseline > $OUT/bench_c3_nobirths.json 2> $OUT/bench_c3_nobirths.err || { tail -5 $OUT/bench_c3_nobirths.err; exit 1; }
for f in bench_c3 bench_c3_nobirths; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', d['value'], 'steps/s; update ms', d['roofline']['avg_kernel_ms'], 'threads/lds/res', d['config']['update_threads'], d['config']['update_lds_bytes'], d['config']['update_resident_workgroups'], 'slow', d['config']['slow_paths'], 'cpu', d.get('cpu_baseline',{}).get('value'))"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c3 -- python3 bench.py --steps 50 --no-cpu-baseline > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { tail -5 $OUT/prof_bench.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
